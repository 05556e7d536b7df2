# Diagnostic variant (scripts/build_variant.sh): the split build in file groups, each group's ORs on the side stream beside the next groups' regions; argument: groups (default 4)
import sys
R = ''  # run in the csrc directory (scripts/build_variant.sh's copy)
G = int(sys.argv[1]) if len(sys.argv) > 1 else 4
FIRST = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0  # > 0: two groups, the first this share of the files
p = R + 'common.h'
s = open(p).read()
old = '''    hipEvent_t fork, join;'''
new = '''    hipEvent_t fork, join;
    hipEvent_t grp[4];  // the .sst build's file groups (region writer -> its ORs)'''
assert old in s; s = s.replace(old, new); open(p, 'w').write(s)
p = R + 'api.hip'
s = open(p).read()
old = '''    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->join, hipEventDisableTiming);'''
new = '''    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->join, hipEventDisableTiming);
    for (int g = 0; g < 4 && e == hipSuccess; g++) e = hipEventCreateWithFlags(&c->grp[g], hipEventDisableTiming);'''
assert old in s; s = s.replace(old, new)
old = '''        if (ctx->join) (void)hipEventDestroy(ctx->join);'''
new = '''        for (int g = 0; g < 4; g++)
            if (ctx->grp[g]) (void)hipEventDestroy(ctx->grp[g]);
        if (ctx->join) (void)hipEventDestroy(ctx->join);'''
assert old in s; s = s.replace(old, new)
open(p, 'w').write(s)

p = R + 'encode.hip'
s = open(p).read()
# SstArgs: file base of the launch
old = '''    uint32_t skip_v;  // the V region is written from value views (lsm_build_sst_views)'''
new = '''    uint32_t skip_v;  // the V region is written from value views (lsm_build_sst_views)
    uint32_t f_base;  // sst_regions_kernel: file of blockIdx.x = f_base + blockIdx.x'''
assert old in s; s = s.replace(old, new)
old = '''    constexpr uint32_t BD = WithV ? kRegBufDwords : kRegIdxDwords;
    __shared__ __attribute__((aligned(16))) uint32_t lds[kRegWaves][BD + kGatherMaskWords];
    const uint32_t f = blockIdx.x;'''
new = '''    constexpr uint32_t BD = WithV ? kRegBufDwords : kRegIdxDwords;
    __shared__ __attribute__((aligned(16))) uint32_t lds[kRegWaves][BD + kGatherMaskWords];
    const uint32_t f = a.f_base + blockIdx.x;'''
assert old in s; s = s.replace(old, new)
old = '''    uint32_t split;     // slice 0 = bits [0, split), slice 1 = [split, m)
    uint32_t nfiles;'''
new = '''    uint32_t split;     // slice 0 = bits [0, split), slice 1 = [split, m)
    uint32_t f_base, nfiles;  // the launch's files: [f_base, f_base + nfiles)'''
assert old in s; s = s.replace(old, new)
old = '''    const uint32_t b = blockIdx.x, f = (b / 16) * 8 + b % 8, sl = (b / 8) % 2;
    if (f >= a.nfiles) return;'''
new = '''    const uint32_t b = blockIdx.x, fl = (b / 16) * 8 + b % 8, sl = (b / 8) % 2;
    if (fl >= a.nfiles) return;
    const uint32_t f = a.f_base + fl;'''
assert old in s; s = s.replace(old, new)
old = '''    a.skip_v = views != nullptr;
    a.hrec = nullptr;'''
new = '''    a.skip_v = views != nullptr;
    a.f_base = 0;
    a.hrec = nullptr;'''
assert old in s; s = s.replace(old, new)
# launches
old = '''    if (chunks) {
        const uint32_t rspans = (max_file_records + kRegSpanRecs - 1) / kRegSpanRecs;
        if (a.skip_v)
            hipLaunchKernelGGL(sst_regions_kernel<false>, dim3(nfile, rspans), dim3(kRegWaves * kWave), 0, rs, a);
        else
            hipLaunchKernelGGL(sst_regions_kernel<true>, dim3(nfile, rspans), dim3(kRegWaves * kWave), 0, rs, a);
        LSM_TRY(hipGetLastError());'''
new = '''    // The split build's ORs of a file need only that file's hash records:
    // the region writer runs in kOrGroups file groups on the caller's stream
    // and each group's ORs follow it on the side stream, beside the next
    // groups' regions (the last group's ORs are the only ones left after the
    // regions: one dispatch round instead of two)
    const uint32_t ngrp = split && !views && !forked && chunks && nfile >= 2 * kOrGroups ? kOrGroups : 1;
    const uint32_t rspans = (max_file_records + kRegSpanRecs - 1) / kRegSpanRecs;
    auto regions = [&](uint32_t f0, uint32_t nf) {
        SstArgs ag = a;
        ag.f_base = f0;
        if (a.skip_v)
            hipLaunchKernelGGL(sst_regions_kernel<false>, dim3(nf, rspans), dim3(kRegWaves * kWave), 0, rs, ag);
        else
            hipLaunchKernelGGL(sst_regions_kernel<true>, dim3(nf, rspans), dim3(kRegWaves * kWave), 0, rs, ag);
    };
    if (chunks && ngrp == 1) {
        regions(0, nfile);
        LSM_TRY(hipGetLastError());'''
assert old in s; s = s.replace(old, new)
old = '''    if (rc == 0 && !split) {
        hipLaunchKernelGGL(sst_meta_kernel, dim3(nfile), dim3(kWave), 0, rs, a);
        LSM_TRY(hipGetLastError());
    } else if (rc == 0) {
        BloomOrArgs bo{};'''
new = '''    if (rc == 0 && !split) {
        hipLaunchKernelGGL(sst_meta_kernel, dim3(nfile), dim3(kWave), 0, rs, a);
        LSM_TRY(hipGetLastError());
    } else if (rc == 0) {
        BloomOrArgs bo{};'''
assert old in s; s = s.replace(old, new)
old = '''        bo.nfiles = nfile;
        hipLaunchKernelGGL(bloom_or_kernel, dim3((nfile + 7) / 8 * 16), dim3(1024), (size_t)(osb / 8), s,
                           bo, a);
        LSM_TRY(hipGetLastError());
    }
    if (forked || vfork) {  // join (also after an error): the caller's stream waits for the side'''
new = '''        auto ors = [&](uint32_t f0, uint32_t nf, hipStream_t os) {
            BloomOrArgs bg = bo;
            bg.f_base = f0;
            bg.nfiles = nf;
            hipLaunchKernelGGL(bloom_or_kernel, dim3((nf + 7) / 8 * 16), dim3(1024), (size_t)(osb / 8), os,
                               bg, a);
        };
        if (ngrp == 1) {
            ors(0, nfile, s);
        } else {
            for (uint32_t g = 0; g < ngrp && rc == 0; g++) {
                const uint32_t f0 = (uint32_t)((uint64_t)nfile * g / ngrp);
                const uint32_t f1 = (uint32_t)((uint64_t)nfile * (g + 1) / ngrp);
                regions(f0, f1 - f0);
                LSM_TRY(hipGetLastError());
                LSM_TRY(hipEventRecord(ctx->grp[g], s));
                LSM_TRY(hipStreamWaitEvent(ctx->side, ctx->grp[g], 0));
                ors(f0, f1 - f0, ctx->side);
                LSM_TRY(hipGetLastError());
            }
        }
        LSM_TRY(hipGetLastError());
    }
    if (forked || vfork || ngrp > 1) {  // join (also after an error): the caller's stream waits for the side'''
assert old in s; s = s.replace(old, new)
old = '''constexpr uint32_t kOrSlices = 2;  // bloom_or_kernel workgroups per filter'''
new = '''constexpr uint32_t kOrSlices = 2;  // bloom_or_kernel workgroups per filter
constexpr uint32_t kOrGroups = %d;  // file groups of the split build (<= lsm_ctx::grp)''' % G
assert old in s; s = s.replace(old, new)
open(p, 'w').write(s)
print('ok', G)
if FIRST > 0:  # two unequal groups: the first FIRST of the files, then the rest
    s = open(p).read()
    old = '''                const uint32_t f0 = (uint32_t)((uint64_t)nfile * g / ngrp);
                const uint32_t f1 = (uint32_t)((uint64_t)nfile * (g + 1) / ngrp);'''
    new = '''                const uint32_t cut = (uint32_t)((double)nfile * %f);
                const uint32_t f0 = g == 0 ? 0u : cut, f1 = g == 0 ? cut : nfile;''' % FIRST
    assert old in s
    s = s.replace(old, new)
    open(p, 'w').write(s)
    print('first', FIRST)
