// common.h — shared device helpers for the gfx950 block codec kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lsm_gpu.h"

#define LSM_HIP_CHECK(expr)                                 \
    do {                                                    \
        hipError_t _e = (expr);                             \
        if (_e != hipSuccess) return -(1000 + (int)_e);     \
    } while (0)

// One context per device and caller thread (include/lsm_gpu.h): the device,
// its CU count, and a side stream with fork / join events for a call that
// runs two independent kernels at once (lsm_build_sst: the VALU-bound filters
// beside the HBM-bound regions, co-resident on the CUs).
// It also owns a small pinned host buffer for the merge's read-backs (its key
// statistics and counts): a copy into pageable memory goes through a staging
// handshake that left 25-55 us idle gaps around each read-back.
struct lsm_ctx {
    int device;
    int num_cus;
    hipStream_t side;
    hipEvent_t fork, join;
    void *host_rb;  // kHostReadback bytes of pinned host memory
    // grow-only pinned host buffer for LSM_TIE_GOHEAP's rank read-back and
    // pop-order upload (pageable copies staged through the runtime: slower)
    void *host_big;
    size_t host_big_bytes;
    // LSM_TIE_GOHEAP calls that replayed the heap (keys with duplicates;
    // distinct keys skip the replay): lsm_goheap_replays
    uint64_t goheap_replays;
};
constexpr size_t kHostReadback = 256 * 1024;

namespace lsm {

constexpr int kWave = 64;
constexpr uint32_t kKeyCap = 1u << 20;  // kv.go:84
constexpr uint32_t kValCap = 1u << 30;  // kv.go:102
// Buffer-resource dword3 for gfx950 raw (stride 0) byte-addressed buffers.
constexpr int kRsrcFlags = 0x00020000;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & (kWave - 1); }

// Global-memory views.  A pointer rebuilt from an integer loses the
// compiler's address-space inference and is accessed with FLAT instructions,
// which also count in lgkmcnt: every later LDS wait would wait for them.
template <class T>
using gptr_t = __attribute__((address_space(1))) T *;
template <class T>
__device__ __forceinline__ gptr_t<T> gbl(T *p) {
    return (gptr_t<T>)p;
}
template <class T>
__device__ __forceinline__ gptr_t<T> gbl_at(uintptr_t a) {
    return (gptr_t<T>)reinterpret_cast<T *>(a);
}

// Wave-uniform value: lets hipcc keep it in an SGPR (T20 in the HIP guide).
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
    uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (uint64_t)hi << 32 | lo;
}

// XCD-contiguous unit order.  Workgroups are dealt round-robin over the 8
// XCDs (observed placement, MI355X_MICROARCH.md "Workgroup dispatch"): WG i
// runs on the XCD of i % 8.  Mapping WG i to unit xcd_linear(i, n) gives each
// XCD one contiguous eighth of the units, so the per-unit metadata lines and
// the partial output lines of neighbouring units meet in one XCD's L2
// instead of being fetched (and written back) by all eight.  A bijection on
// [0, n) for any n; correctness never depends on the placement.
__device__ __forceinline__ uint32_t xcd_linear(uint32_t i, uint32_t n) {
    const uint32_t q = n >> 3, r = n & 7, x = i & 7, k = i >> 3;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
}

// Raw buffer over [base, base+bytes): loads past `bytes` return 0 and touch no memory.
__device__ __forceinline__ rsrc_t make_rsrc(const void *base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)bytes,
                                             kRsrcFlags);
}

__device__ __forceinline__ u32x4 ld_b128(rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}
__device__ __forceinline__ uint32_t ld_b32(rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
}

// Bytes [s, s+4) of a little-endian byte stream given the two aligned dwords
// that cover them.
__device__ __forceinline__ uint32_t funnel(uint32_t lo, uint32_t hi, uint32_t s) {
    return __builtin_amdgcn_alignbyte(hi, lo, s & 3);
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// Number of set bits of m in the lanes below this one.
__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

// Wave-64 inclusive prefix sums with DPP row shifts (1, 2, 4, 8 within a
// 16-lane row) and the gfx9 row broadcasts (lane 15 -> next row, lane 31 ->
// upper half): six VALU moves, no LDS round trip (a __shfl_up scan is six
// ds_bpermute waits).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const uint32_t l = lane_id(), rl = l & 15;
    uint32_t t;
    t = dpp_mov<0x111>(v); v += rl >= 1 ? t : 0;   // row_shr:1
    t = dpp_mov<0x112>(v); v += rl >= 2 ? t : 0;   // row_shr:2
    t = dpp_mov<0x114>(v); v += rl >= 4 ? t : 0;   // row_shr:4
    t = dpp_mov<0x118>(v); v += rl >= 8 ? t : 0;   // row_shr:8
    t = dpp_mov<0x142>(v); v += (l & 31) >= 16 ? t : 0;  // row_bcast:15
    t = dpp_mov<0x143>(v); v += l >= 32 ? t : 0;   // row_bcast:31
    return v;
}

__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t v) {
    const uint32_t l = lane_id(), rl = l & 15;
#define LSM_SCAN64_STEP(CTRL, COND)                                                     \
    {                                                                                  \
        const uint64_t t = (uint64_t)dpp_mov<CTRL>((uint32_t)(v >> 32)) << 32 |        \
                           dpp_mov<CTRL>((uint32_t)v);                                 \
        v += (COND) ? t : 0;                                                           \
    }
    LSM_SCAN64_STEP(0x111, rl >= 1)
    LSM_SCAN64_STEP(0x112, rl >= 2)
    LSM_SCAN64_STEP(0x114, rl >= 4)
    LSM_SCAN64_STEP(0x118, rl >= 8)
    LSM_SCAN64_STEP(0x142, (l & 31) >= 16)
    LSM_SCAN64_STEP(0x143, l >= 32)
#undef LSM_SCAN64_STEP
    return v;
}

// Exclusive wave prefix sum (64 lanes); *total = the sum over all lanes.
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t *total) {
    const uint32_t inc = wave_incl_scan(v);
    *total = (uint32_t)__builtin_amdgcn_readlane((int)inc, kWave - 1);
    return inc - v;
}

__device__ __forceinline__ uint64_t wave_excl_scan64(uint64_t v, uint64_t *total) {
    const uint64_t inc = wave_incl_scan64(v);
    *total = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(inc >> 32), kWave - 1) << 32 |
             (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)inc, kWave - 1);
    return inc - v;
}

// Copy `len` bytes from buffer offset `src` (rsrc-relative, any alignment)
// to global `dst` (any alignment) with the whole wave: interior dwords by
// dword stores, the <=3 edge bytes at each end by byte stores.  Requires
// src >= 3: the first dword is read from src - (dst & 3), and a wrapped
// offset plus the folded +4 of the next dword reads as out of range (0).
__device__ __forceinline__ void wave_copy(rsrc_t r, uint32_t src, uint8_t *dst, uint32_t len) {
    if (len == 0) return;
    uintptr_t d0 = reinterpret_cast<uintptr_t>(dst);
    uint32_t head = (uint32_t)(d0 & 3);
    gptr_t<uint32_t> dA = gbl_at<uint32_t>(d0 - head);
    uint32_t ndw = (head + len + 3) >> 2;
    for (uint32_t j = lane_id(); j < ndw; j += kWave) {
        uint32_t S = src - head + 4 * j;  // may wrap below 0: OOB loads return 0
        uint32_t Sa = S & ~3u;
        uint32_t v = funnel(ld_b32(r, Sa), ld_b32(r, Sa + 4), S);
        uint32_t lo_b = (j == 0) ? head : 0;
        uint32_t end = head + len - 4 * j;
        uint32_t hi_b = end < 4 ? end : 4;
        if (lo_b == 0 && hi_b == 4) {
            dA[j] = v;
        } else {
            gptr_t<uint8_t> db = (gptr_t<uint8_t>)(dA + j);
            for (uint32_t t = lo_b; t < hi_b; t++) db[t] = (uint8_t)(v >> (8 * t));
        }
    }
}

}  // namespace lsm
