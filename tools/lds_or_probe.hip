// lds_or_probe.hip — LDS bit-set throughput on gfx950 (tools only, never the
// product): what rate can a workgroup OR scattered bits into an LDS bitmap at,
// the operation bloom_or_kernel spends its time in.  Every thread makes `per`
// pseudo-random bit positions (splitmix-style hash of its id) over `span`
// bits and, per mode:
//   0  ds_or_b32 of every position                    (all lanes active)
//   1  ds_or_b32 only of positions inside the lower half of span (the
//      current kernel's shape: about half the lanes of each instruction)
//   2  ds_or_b32 with the word's bank forced to lane & 31 (conflict-free)
//   3  ds_write_b32 of every position (no read-modify-write; wrong bits)
//   4  no LDS op: the positions' VALU cost only
//   5  as 1, but the in-slice positions of 2 rounds compacted (ballot +
//      mbcnt) through a per-wave LDS queue, ORed by full-lane instructions
//   6  as 0, with ds_or_b64 (bit in a 64-bit word)
//   7  LDS bounds check: every lane stores ~0 past the allocation and reads
//      it back (0 if the hardware drops out-of-range accesses)
//   8  as 1, the out-of-slice lanes' ORs left to the bounds check (address
//      past the allocation), no exec mask
//   9  as 1, branch-free: OR of 0 into an in-range word for out-of-slice lanes
// The bitmap is stored to `out` at the end so no mode is dead code.
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

template <int MODE>
__global__ __launch_bounds__(1024) void lds_or_kernel(uint32_t span, uint32_t per, uint32_t *out) {
    extern __shared__ __attribute__((aligned(16))) uint32_t bits[];
    const uint32_t tot = MODE == 1 || MODE == 5 || MODE == 8 || MODE == 9 ? (span / 2 + 31) / 32
                                                                          : (span + 31) / 32 + 64;
    __shared__ uint32_t q[16][256];
    for (uint32_t i = threadIdx.x; i < tot; i += blockDim.x) bits[i] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t seed = (blockIdx.x * 1024 + threadIdx.x) * 0x9e3779b9u;
    const uint32_t half = span / 2;
    uint32_t acc = 0, qn = 0;
    uint32_t r = mix32(seed);
    if (MODE == 7) {
        const uint32_t a = tot + threadIdx.x;  // past the allocation
        bits[a] = ~0u;
        __syncthreads();
        out[blockIdx.x * 1024 + threadIdx.x] = bits[a];
        return;
    }
    for (uint32_t i = 0; i < per; i++) {
        r = r * 1664525u + 1013904223u;  // cheap positions: VALU must not bound the probe
        const uint32_t p = __umulhi(r, span);
        if (MODE == 0) {
            atomicOr(&bits[p >> 5], 1u << (p & 31));
        } else if (MODE == 1) {
            if (p < half) atomicOr(&bits[p >> 5], 1u << (p & 31));
        } else if (MODE == 2) {
            atomicOr(&bits[((p >> 5) & ~31u) | (lane & 31)], 1u << (p & 31));
        } else if (MODE == 3) {
            bits[p >> 5] = 1u << (p & 31);
        } else if (MODE == 4) {
            acc ^= p;
        } else if (MODE == 5) {
            const bool in = p < half;
            const uint64_t b = __ballot(in);
            const uint32_t before = __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0));
            if (in) q[w][qn + before] = p;
            qn += (uint32_t)__builtin_popcountll(b);
            if (qn >= 64 * 2) {  // two full rounds queued: OR them with all lanes
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                for (uint32_t t = 0; t < 2; t++) {  // the oldest 128 entries, [0, 128)
                    const uint32_t x = q[w][64 * t + lane];
                    atomicOr(&bits[x >> 5], 1u << (x & 31));
                }
                qn -= 128;
                // the leftover entries [128, 128 + qn) move to the front
                const uint32_t left = qn;
                uint32_t v = 0;
                if (lane < left) v = q[w][128 + lane];
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                if (lane < left) q[w][lane] = v;
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            }
        } else if (MODE == 8) {
            // p >= half: word index >= the allocation, dropped by the bounds check
            __hip_atomic_fetch_or(&bits[p >> 5], 1u << (p & 31), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP);
        } else if (MODE == 9) {
            const uint32_t w5 = p >> 5, nwd = half >> 5;
            const uint32_t wd = min(w5, w5 - nwd);  // folded into range
            atomicOr(&bits[wd], p < half ? 1u << (p & 31) : 0u);
        } else if (MODE == 6) {
            atomicOr(reinterpret_cast<unsigned long long *>(&bits[(p >> 6) * 2]), 1ull << (p & 63));
        }
    }
    if (MODE == 5 && lane < qn) {
        const uint32_t x = q[w][lane];
        atomicOr(&bits[x >> 5], 1u << (x & 31));
    }
    __syncthreads();
    uint32_t x = acc;
    for (uint32_t i = threadIdx.x; i < tot; i += blockDim.x) x ^= bits[i];
    out[blockIdx.x * 1024 + threadIdx.x] = x;
}

typedef void (*kfn)(uint32_t, uint32_t, uint32_t *);

extern "C" int lds_or_probe(int mode, uint32_t grid, uint32_t threads, uint32_t span, uint32_t per,
                            void *out, void *stream) {
    const uint32_t half = span / 2;
    const bool sl = mode == 1 || mode == 5 || mode == 8 || mode == 9;
    const size_t lds = 4ull * (sl ? (half + 31) / 32 : (span + 31) / 32 + 64);
    hipStream_t s = (hipStream_t)stream;
    uint32_t *o = (uint32_t *)out;
#define L(M) hipLaunchKernelGGL(lds_or_kernel<M>, dim3(grid), dim3(threads), lds, s, span, per, o)
    switch (mode) {
        case 0: L(0); break;
        case 1: L(1); break;
        case 2: L(2); break;
        case 3: L(3); break;
        case 4: L(4); break;
        case 5: L(5); break;
        case 6: L(6); break;
        case 7: L(7); break;
        case 8: L(8); break;
        case 9: L(9); break;
        default: return -1;
    }
#undef L
    return (int)hipGetLastError();
}
