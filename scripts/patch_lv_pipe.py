# A/B variant (scripts/build_variant.sh): the level search with fewer dependent global
# latencies.  lv_classify_kernel: the table prefixes are staged after the key loads are
# issued; both probes' searches run before their candidate tables' fields are loaded
# (both loads in flight together, the hashes computed under them); the slot stores use
# the fields already in registers.  lv_test_kernel: the table's grid row is staged in LDS
# beside its counts, so locating a probe's slot is LDS-only.
s = open('encode.hip').read()

# ---- test kernel: grid row in LDS
old = '''    __shared__ uint32_t sb[kLvMaxWgs + 1];  // first probe of each workgroup's segment
    __shared__ uint32_t part[kLvThreads];
    const uint32_t f = blockIdx.x, t = threadIdx.x;
    // the table's segments: counts scanned (nwg <= 1,024: one per thread)
    const uint32_t c = t < nwg ? w.cnt[(uint64_t)f * nwg + t] : 0u;
    part[t] = c;'''
assert old in s
s = s.replace(old, '''    __shared__ uint32_t sb[kLvMaxWgs + 1];  // first probe of each workgroup's segment
    __shared__ uint32_t sg[kLvMaxWgs];      // its first slot in that workgroup
    __shared__ uint32_t part[kLvThreads];
    const uint32_t f = blockIdx.x, t = threadIdx.x;
    // the table's segments: counts scanned (nwg <= 1,024: one per thread)
    const uint32_t c = t < nwg ? w.cnt[(uint64_t)f * nwg + t] : 0u;
    if (t < nwg) sg[t] = w.grid[(uint64_t)f * nwg + t];
    part[t] = c;''')
old = '''        return (uint64_t)a * kLvProbes + w.grid[(uint64_t)f * nwg + a] + (q - sb[a]);'''
assert old in s
s = s.replace(old, '''        return (uint64_t)a * kLvProbes + sg[a] + (q - sb[a]);''')

# ---- classify kernel: new body
import os
if os.environ.get('LV_PART') == 'grid':
    open('encode.hip', 'w').write(s)
    print('ok (grid only)')
    raise SystemExit(0)
b = s.index('__global__ __launch_bounds__(kLvThreads) void lv_classify_kernel(')
e = s.index('// The filter words of F: the first `cap` bytes into LDS')
new = r'''__global__ __launch_bounds__(kLvThreads) void lv_classify_kernel(const uint8_t *img, uint32_t nfile,
                                                                 const uint8_t *keys, const uint64_t *koff,
                                                                 uint64_t k_begin, uint64_t nkeys, LvWs w,
                                                                 uint32_t nwg, int32_t *table,
                                                                 uint8_t *may) {
    __shared__ uint4 slo[kLvMaxFiles];
    __shared__ uint32_t lh[kLvMaxFiles];
    __shared__ uint32_t part[kLvThreads];
    const uint32_t t = threadIdx.x;
    uint64_t k0[kLvPer], kl[kLvPer], f0[kLvPer], f1[kLvPer];
#pragma unroll
    for (uint32_t p = 0; p < kLvPer; p++) {
        const uint64_t i = k_begin + (uint64_t)blockIdx.x * kLvProbes + p * kLvThreads + t;
        k0[p] = i < nkeys ? koff[i] : 0;
        kl[p] = i < nkeys ? koff[i + 1] - k0[p] : 0;
    }
#pragma unroll
    for (uint32_t p = 0; p < kLvPer; p++) {
        const uint64_t i = k_begin + (uint64_t)blockIdx.x * kLvProbes + p * kLvThreads + t;
        f0[p] = i < nkeys ? ldg_u64_unaligned(keys + k0[p]) : 0;
        f1[p] = i < nkeys ? ldg_u64_unaligned(keys + k0[p] + 8) : 0;
    }
    // the prefixes behind the key loads (both latencies overlap)
    for (uint32_t f = t; f < nfile; f += kLvThreads) {
        const McFile &F = w.files[f];
        slo[f] = make_uint4(F.lo[0], F.lo[1], F.lo[2], F.lo[3]);
        lh[f] = 0;
    }
    uint32_t kw[kLvPer][4];
#pragma unroll
    for (uint32_t p = 0; p < kLvPer; p++) {
        const uint64_t l = kl[p];
        if (l < 8) { f0[p] &= l ? (~0ull >> (64 - 8 * l)) : 0; f1[p] = 0; }
        else if (l < 16) f1[p] &= l > 8 ? (~0ull >> (128 - 8 * l)) : 0;
        kw[p][0] = __builtin_bswap32((uint32_t)f0[p]);
        kw[p][1] = __builtin_bswap32((uint32_t)(f0[p] >> 32));
        kw[p][2] = __builtin_bswap32((uint32_t)f1[p]);
        kw[p][3] = __builtin_bswap32((uint32_t)(f1[p] >> 32));
    }
    __syncthreads();
    auto lo_lds = [&](uint32_t h, uint32_t bw[4]) {
        const uint4 v = slo[h];
        bw[0] = v.x; bw[1] = v.y; bw[2] = v.z; bw[3] = v.w;
    };
    // 1. both searches (LDS)
    uint32_t lo[kLvPer], idx[kLvPer];
#pragma unroll
    for (uint32_t p = 0; p < kLvPer; p++) {
        const uint64_t i = k_begin + (uint64_t)blockIdx.x * kLvProbes + p * kLvThreads + t;
        lo[p] = 0;
        if (i < nkeys) lo[p] = lv_search(nfile, lo_lds, w.files, img, kw[p], kl[p], keys + k0[p]);
        idx[p] = lo[p] ? lo[p] - 1 : 0;  // manager.go:189-191
        if (i < nkeys) table[i] = (int32_t)idx[p];
    }
    // 2. both candidates' fields in flight, the hashes computed under them
    uint32_t hi[kLvPer][4], hl[kLvPer], ok[kLvPer], fk[kLvPer];
    uint64_t hat[kLvPer], fm[kLvPer], fmr[kLvPer];
#pragma unroll
    for (uint32_t p = 0; p < kLvPer; p++) {
        const McFile &F = w.files[idx[p]];
        for (int j = 0; j < 4; j++) hi[p][j] = F.hi[j];
        hl[p] = F.hi_len; ok[p] = F.ok; fk[p] = F.k;
        hat[p] = F.hi_at; fm[p] = F.m; fmr[p] = F.mr;
    }
    uint64_t hh[kLvPer][4];
#pragma unroll
    for (uint32_t p = 0; p < kLvPer; p++) sum256_pre(keys + k0[p], kl[p], f0[p], f1[p], hh[p]);
    // 3. MayContain's range check (sstable.go:301): lo > 0 means f(lo - 1) was
    // evaluated false, i.e. MinKey <= key; then MaxKey >= key and a decoded filter
    uint32_t cand[kLvPer], rank[kLvPer];
#pragma unroll
    for (uint32_t p = 0; p < kLvPer; p++) {
        const uint64_t i = k_begin + (uint64_t)blockIdx.x * kLvProbes + p * kLvThreads + t;
        cand[p] = kMcNone;
        if (i >= nkeys) continue;
        bool test = false;
        if (lo[p] > 0 && ok[p]) {
            int r = prefix_cmp(hi[p], kw[p]);
            if (r == 0) r = bound_cmp(hi[p], hl[p], img + hat[p], kw[p], kl[p], keys + k0[p]);
            test = r >= 0;
        }
        if (!test) {
            may[i] = 0;
            continue;
        }
        cand[p] = idx[p];
        rank[p] = atomicAdd(&lh[idx[p]], 1u);
    }
    __syncthreads();
    // exclusive scan of the per-table counts (<= 2,048 tables, 2 per thread)
    const uint32_t c0 = 2 * t < nfile ? lh[2 * t] : 0u, c1 = 2 * t + 1 < nfile ? lh[2 * t + 1] : 0u;
    part[t] = c0 + c1;
    __syncthreads();
    for (uint32_t d = 1; d < kLvThreads; d <<= 1) {
        const uint32_t x = t >= d ? part[t - d] : 0u;
        __syncthreads();
        part[t] += x;
        __syncthreads();
    }
    const uint32_t ex = part[t] - c0 - c1;
    __syncthreads();  // every lh read before it is overwritten with offsets
    if (2 * t < nfile) {
        lh[2 * t] = ex;
        w.grid[(uint64_t)(2 * t) * nwg + blockIdx.x] = ex;
        w.cnt[(uint64_t)(2 * t) * nwg + blockIdx.x] = c0;
    }
    if (2 * t + 1 < nfile) {
        lh[2 * t + 1] = ex + c0;
        w.grid[(uint64_t)(2 * t + 1) * nwg + blockIdx.x] = ex + c0;
        w.cnt[(uint64_t)(2 * t + 1) * nwg + blockIdx.x] = c1;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t p = 0; p < kLvPer; p++) {
        if (cand[p] == kMcNone) continue;
        const uint64_t i = k_begin + (uint64_t)blockIdx.x * kLvProbes + p * kLvThreads + t;
        const uint64_t slot = (uint64_t)blockIdx.x * kLvProbes + lh[cand[p]] + rank[p];
        w.ids[slot] = (uint32_t)(i - k_begin);
        if (fm[p] != 0 && fm[p] <= (1ull << kHashRecBits) && fk[p] <= kSplitMaxK) {  // lv_compact
            store_hash_rec(hh[p], (uint32_t)fm[p], (uint32_t)fmr[p], (uint32_t)(fmr[p] >> 32),
                           reinterpret_cast<uint32_t *>(w.rec + slot));
        } else {
            *(gptr_t<u64x2>)gbl(w.rec + slot) = u64x2{hh[p][0], hh[p][1]};
            *(gptr_t<u64x2>)gbl(w.ext + slot) = u64x2{hh[p][2], hh[p][3]};
        }
    }
}

'''
s = s[:b] + new + s[e:]
open('encode.hip', 'w').write(s)
print('ok')
