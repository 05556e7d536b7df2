# A/B variant: the two classify kernels (mc_classify_kernel, lv_classify_kernel) with their
# loads in flight together: the key offsets loaded unconditionally at a clamped index (a
# load under a branch whose join waits for it serializes the probes), the table fill
# after the key loads (its LDS stores no longer hold the key loads back), and in the
# level search both probes' candidate fields loaded before either range check.
s = open('encode.hip').read()

# ---- key offsets: clamped, unconditional (both kernels)
for per, thr, probes, idx in (('kMcGroupPer', 'kMcGroupThreads', 'kMcGroupProbes',
                               '(uint64_t)blockIdx.x * kMcGroupProbes + p * kMcGroupThreads + threadIdx.x'),
                              ('kLvPer', 'kLvThreads', 'kLvProbes',
                               'k_begin + (uint64_t)blockIdx.x * kLvProbes + p * kLvThreads + t')):
    old = f'''        const uint64_t i = {idx};
        k0[p] = i < nkeys ? koff[i] : 0;
        kl[p] = i < nkeys ? koff[i + 1] - k0[p] : 0;'''
    assert old in s, per
    s = s.replace(old, f'''        const uint64_t i = {idx};
        const uint64_t ic = i < nkeys ? i : nkeys - 1;  // loads not under a branch
        const uint64_t a0 = koff[ic], a1 = koff[ic + 1];
        k0[p] = i < nkeys ? a0 : 0;
        kl[p] = i < nkeys ? a1 - a0 : 0;''')

# ---- mc_classify: the fill after the key loads
old = '''    if (!w.flag[0]) return;
    for (uint32_t f = threadIdx.x; f < nfile; f += kMcGroupThreads) {
        const McFile &F = w.files[f];
        slo[f] = make_uint4(F.lo[0], F.lo[1], F.lo[2], F.lo[3]);
        shi[f] = make_uint4(F.hi[0], F.hi[1], F.hi[2], F.hi[3]);
        lh[f] = 0;
    }
'''
assert old in s
s = s.replace(old, '''    if (!w.flag[0]) return;
''')
old = '''        f1[p] = i < nkeys ? ldg_u64_unaligned(keys + k0[p] + 8) : 0;
    }
    {   // the workgroup's rows of the hit matrix start at 0'''
assert old in s
s = s.replace(old, '''        f1[p] = i < nkeys ? ldg_u64_unaligned(keys + k0[p] + 8) : 0;
    }
    for (uint32_t f = threadIdx.x; f < nfile; f += kMcGroupThreads) {
        const McFile &F = w.files[f];
        slo[f] = make_uint4(F.lo[0], F.lo[1], F.lo[2], F.lo[3]);
        shi[f] = make_uint4(F.hi[0], F.hi[1], F.hi[2], F.hi[3]);
        lh[f] = 0;
    }
    {   // the workgroup's rows of the hit matrix start at 0''')

# ---- lv_classify: the fill after the key loads
old = '''    __shared__ uint32_t part[kLvThreads];
    const uint32_t t = threadIdx.x;
    for (uint32_t f = t; f < nfile; f += kLvThreads) {
        const McFile &F = w.files[f];
        slo[f] = make_uint4(F.lo[0], F.lo[1], F.lo[2], F.lo[3]);
        lh[f] = 0;
    }
'''
assert old in s
s = s.replace(old, '''    __shared__ uint32_t part[kLvThreads];
    const uint32_t t = threadIdx.x;
''')
old = '''        f1[p] = i < nkeys ? ldg_u64_unaligned(keys + k0[p] + 8) : 0;
    }
    uint32_t kw[kLvPer][4];'''
assert old in s
s = s.replace(old, '''        f1[p] = i < nkeys ? ldg_u64_unaligned(keys + k0[p] + 8) : 0;
    }
    for (uint32_t f = t; f < nfile; f += kLvThreads) {
        const McFile &F = w.files[f];
        slo[f] = make_uint4(F.lo[0], F.lo[1], F.lo[2], F.lo[3]);
        lh[f] = 0;
    }
    uint32_t kw[kLvPer][4];''')

# ---- lv_classify: searches, then both candidates' fields, then the checks
b = s.index('''    uint32_t cand[kLvPer], rank[kLvPer];
    uint64_t hh[kLvPer][4];
#pragma unroll
    for (uint32_t p = 0; p < kLvPer; p++) {''')
e = s.index('''    __syncthreads();
    // exclusive scan of the per-table counts (<= 2,048 tables, 2 per thread)''')
new = '''    uint32_t lo[kLvPer], idx[kLvPer];
#pragma unroll
    for (uint32_t p = 0; p < kLvPer; p++) {
        const uint64_t i = k_begin + (uint64_t)blockIdx.x * kLvProbes + p * kLvThreads + t;
        lo[p] = i < nkeys ? lv_search(nfile, lo_lds, w.files, img, kw[p], kl[p], keys + k0[p]) : 0u;
        idx[p] = lo[p] ? lo[p] - 1 : 0;  // manager.go:189-191
        if (i < nkeys) table[i] = (int32_t)idx[p];
    }
    // both candidates' fields in flight before either check
    uint32_t hi[kLvPer][4], hl[kLvPer], ok[kLvPer];
    uint64_t hat[kLvPer];
#pragma unroll
    for (uint32_t p = 0; p < kLvPer; p++) {
        const McFile &F = w.files[idx[p]];
#pragma unroll
        for (int j = 0; j < 4; j++) hi[p][j] = F.hi[j];
        hl[p] = F.hi_len; ok[p] = F.ok; hat[p] = F.hi_at;
    }
    uint32_t cand[kLvPer], rank[kLvPer];
    uint64_t hh[kLvPer][4];
#pragma unroll
    for (uint32_t p = 0; p < kLvPer; p++) {
        const uint64_t i = k_begin + (uint64_t)blockIdx.x * kLvProbes + p * kLvThreads + t;
        cand[p] = kMcNone;
        if (i >= nkeys) continue;
        const uint8_t *kp = keys + k0[p];
        // MayContain (sstable.go:301): lo > 0 means f(lo - 1) was evaluated
        // false, i.e. MinKey <= key; then MaxKey >= key and a decoded filter
        bool test = false;
        if (lo[p] > 0 && ok[p]) {
            int r = prefix_cmp(hi[p], kw[p]);
            if (r == 0) r = bound_cmp(hi[p], hl[p], img + hat[p], kw[p], kl[p], kp);
            test = r >= 0;
        }
        if (!test) {
            may[i] = 0;
            continue;
        }
        cand[p] = idx[p];
        rank[p] = atomicAdd(&lh[idx[p]], 1u);
        sum256_pre(kp, kl[p], f0[p], f1[p], hh[p]);
    }
'''
s = s[:b] + new + s[e:]
open('encode.hip', 'w').write(s)
print('ok cls')
