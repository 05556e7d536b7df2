// murmur.h — device MurmurHash3 sum256 and bloom locations (gfx950).
//
// Device restatement of go-lsm's digest128.sum256 (sstable/bloom/murmur.go:245-275):
// MMH3_x64_128(seed 0) of `key` and of `key || 0x01`, computed in one pass
// over the key (the 16-byte blocks are shared by both digests; only the tail
// differs).  Locations follow bloom.go:133-141; `% m` uses a Barrett
// reduction with a host-precomputed reciprocal (one correction step).
#pragma once

#include "common.h"

namespace lsm {

constexpr uint64_t kMC1 = 0x87c37b91114253d5ull;
constexpr uint64_t kMC2 = 0x4cf5ad432745937full;

__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

__device__ __forceinline__ void mmh3_block(uint64_t &h1, uint64_t &h2, uint64_t k1, uint64_t k2) {
    k1 *= kMC1; k1 = rotl64(k1, 31); k1 *= kMC2; h1 ^= k1;
    h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
    k2 *= kMC2; k2 = rotl64(k2, 33); k2 *= kMC1; h2 ^= k2;
    h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
}

// Tail words (k1 = bytes 0..7, k2 = bytes 8..15 of a tail of tl < 16 bytes),
// then finalization with the total length.
__device__ __forceinline__ void mmh3_final(uint64_t h1, uint64_t h2, uint64_t k1, uint64_t k2,
                                           uint32_t tl, uint64_t len, uint64_t &o1,
                                           uint64_t &o2) {
    if (tl > 8) { k2 *= kMC2; k2 = rotl64(k2, 33); k2 *= kMC1; h2 ^= k2; }
    if (tl > 0) { k1 *= kMC1; k1 = rotl64(k1, 31); k1 *= kMC2; h1 ^= k1; }
    h1 ^= len; h2 ^= len;
    h1 += h2; h2 += h1;
    h1 = fmix64(h1); h2 = fmix64(h2);
    h1 += h2; h2 += h1;
    o1 = h1; o2 = h2;
}

// Unaligned little-endian u32 from global memory (two aligned dword loads).
// Requires the 4 bytes past p+3 to be readable (16-byte padded arenas).
__device__ __forceinline__ uint32_t ldg_u32_unaligned(const uint8_t *p) {
    uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const gptr_t<const uint32_t> w = gbl_at<const uint32_t>(a & ~(uintptr_t)3);
    return funnel(w[0], w[1], (uint32_t)a);
}

__device__ __forceinline__ uint64_t ldg_u64_unaligned(const uint8_t *p) {
    uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const gptr_t<const uint32_t> w = gbl_at<const uint32_t>(a & ~(uintptr_t)3);
    uint32_t s = (uint32_t)a;
    uint32_t x0 = w[0], x1 = w[1], x2 = w[2];
    return (uint64_t)funnel(x1, x2, s) << 32 | funnel(x0, x1, s);
}

// sum256 (murmur.go:245-275) of key[0..len), with the key's first 16 bytes
// already loaded as (f0, f1) (callers prefetch them; bytes past len are
// ignored).  Longer keys load their remaining blocks here.
__device__ __forceinline__ void sum256_pre(const uint8_t *key, uint64_t len, uint64_t f0,
                                           uint64_t f1, uint64_t h[4]) {
    uint64_t h1 = 0, h2 = 0;
    const uint64_t nb = len / 16;
    if (nb) mmh3_block(h1, h2, f0, f1);
    for (uint64_t i = 1; i < nb; i++)
        mmh3_block(h1, h2, ldg_u64_unaligned(key + 16 * i), ldg_u64_unaligned(key + 16 * i + 8));
    const uint32_t tl = (uint32_t)(len & 15);
    uint64_t k1 = 0, k2 = 0;
    if (tl) {
        // Gather the tail bytes; bytes beyond tl are masked off.
        const uint8_t *tail = key + 16 * nb;
        const uint64_t w0 = nb ? ldg_u64_unaligned(tail) : f0;
        const uint64_t w1 = tl > 8 ? (nb ? ldg_u64_unaligned(tail + 8) : f1) : 0;
        k1 = tl >= 8 ? w0 : (w0 & ((1ull << (8 * tl)) - 1));
        k2 = tl > 8 ? (w1 & ((1ull << (8 * (tl - 8))) - 1)) : 0;
    }
    mmh3_final(h1, h2, k1, k2, tl, len, h[0], h[1]);
    // Second digest: virtually append 0x01 at tail position tl.
    if (tl == 15) {
        uint64_t kk2 = k2 | (1ull << 56);
        mmh3_block(h1, h2, k1, kk2);
        mmh3_final(h1, h2, 0, 0, 0, len + 1, h[2], h[3]);
    } else {
        uint64_t kk1 = k1, kk2 = k2;
        if (tl < 8) kk1 |= 1ull << (8 * tl);
        else kk2 |= 1ull << (8 * (tl - 8));
        mmh3_final(h1, h2, kk1, kk2, tl + 1, len + 1, h[2], h[3]);
    }
}

// sum256 of key[0..len).  Reads up to 16 bytes past short keys (batches are
// 16-byte padded, include/lsm_gpu.h).
__device__ __forceinline__ void sum256(const uint8_t *key, uint64_t len, uint64_t h[4]) {
    sum256_pre(key, len, ldg_u64_unaligned(key), ldg_u64_unaligned(key + 8), h);
}

// location(h, i) before the modulo (bloom.go:133-136).  Scalar arguments:
// selecting among array elements by a runtime index would spill the digest
// to scratch.
__device__ __forceinline__ uint64_t location(uint64_t h0, uint64_t h1, uint64_t h2, uint64_t h3,
                                             uint32_t i) {
    const uint32_t m4 = i & 3;
    const uint64_t a = (m4 & 1) ? h1 : h0;
    const uint64_t b = (m4 == 0 || m4 == 3) ? h2 : h3;
    return a + (uint64_t)i * b;
}

// x mod m with Barrett reciprocal r = floor((2^64-1)/m) (m < 2^63).
__device__ __forceinline__ uint64_t mod_barrett(uint64_t x, uint64_t m, uint64_t r) {
    uint64_t q = __umul64hi(x, r);
    uint64_t rem = x - q * m;
    return rem >= m ? rem - m : rem;
}

// x mod m for m <= 2^30 in 32-bit arithmetic, r = floor((2^64-1)/m) split
// as (rh, rl).  hi64(x*r) is in [q-1, q] (q = floor(x/m)); dropping the low
// partial product and the carries of the middle ones costs at most 2 more,
// so q' = the low 32 bits of xh*rh + hi(xh*rl) + hi(xl*rh) (mod 2^32) is in
// [q-3, q] and x - q'*m, which is < 4m <= 2^32, is exact in 32 bits; three
// conditional subtractions finish it (v_sub + v_min each).
__device__ __forceinline__ uint32_t mod_small(uint64_t x, uint32_t m, uint32_t rl, uint32_t rh) {
    const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
    const uint32_t q = xh * rh + __umulhi(xh, rl) + __umulhi(xl, rh);
    uint32_t rem = xl - q * m;
    rem = min(rem, rem - m);
    rem = min(rem, rem - m);
    rem = min(rem, rem - m);
    return rem;
}

}  // namespace lsm
