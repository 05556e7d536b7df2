# A/B variant: scripts/patch_lv_grid.py plus filter_test_rec with every bit read of a
# probe issued before any is waited for (the LDS reads at clamped addresses, the tail reads
# under a predicate into their own registers), instead of one branch per location whose
# join waits for its load (sixteen serialized round trips per probe).
import os
os.environ['LV_PART'] = 'grid'
try:
    exec(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'patch_lv_pipe.py')).read())
except SystemExit:
    pass
s = open('encode.hip').read()
b = s.index('__device__ __forceinline__ uint32_t filter_test_rec(')
e = s.index('__global__ __launch_bounds__(kLvThreads) void lv_test_kernel(')
new = r'''__device__ __forceinline__ uint32_t filter_test_rec(const McFile &F, const HashRecSteps &H0,
                                                    uint32_t m, const uint8_t *lb, uint64_t in_lds,
                                                    const uint8_t *src) {
    uint32_t r[4] = {H0.r[0], H0.r[1], H0.r[2], H0.r[3]};
    uint32_t pos[kSplitMaxK];
#pragma unroll
    for (uint32_t j = 0; j < kSplitMaxK; j++) {
        const uint32_t c = j & 3, n = j >> 2;
        pos[j] = r[c];
        if (n < 3) {
            const uint32_t t = r[c] + H0.st[c][n];
            r[c] = min(t, t - m);
        }
    }
    // all reads in flight: LDS at a clamped address, the tail past the LDS
    // copy (through L2) only where a live location falls in it
    uint32_t lv[kSplitMaxK], gv[kSplitMaxK];
#pragma unroll
    for (uint32_t j = 0; j < kSplitMaxK; j++) {
        const uint32_t p = pos[j];
        const uint32_t q = 8 * (p >> 6) + 7 - ((p & 63) >> 3);
        const bool inl = q < in_lds;
        lv[j] = lb[inl ? q : 0u];
        gv[j] = 0xFFu;
        if (j < F.k && !inl && p < F.nbits) gv[j] = gbl(src)[q];
    }
    uint32_t bits = 1;
#pragma unroll
    for (uint32_t j = 0; j < kSplitMaxK; j++) {
        const uint32_t p = pos[j];
        const uint32_t q = 8 * (p >> 6) + 7 - ((p & 63) >> 3);
        const uint32_t byte = q < in_lds ? lv[j] : gv[j];
        // bitset.Test is false past its length
        const uint32_t bit = p < F.nbits ? (byte >> (p & 7)) & 1u : 0u;
        bits &= j < F.k ? bit : 1u;
    }
    return bits;
}

'''
s = s[:b] + new + s[e:]
open('encode.hip', 'w').write(s)
print('ok bits')
