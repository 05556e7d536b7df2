// merge.hip — the compaction merge on the GPU.
//
// CompactAndMergeKVs (sstable/merge.go:42-94) pushes every pair into a
// container/heap, pops them in key order and, per pop: skips a key equal to
// the last written one (when that key is non-empty), drops tombstones when
// the target level is maxSSTableLevel (6), adds the pair to the builder,
// flushes a file once EstimateSize sums reach 2 MiB (builder.go:34-42) and
// forgets the last written key at every flush.
//
// Tie order: container/heap is not stable, so the pop order of equal keys is
// whatever the heap's array history makes it (about one duplicate group in
// seven differs from input order on compaction-shaped inputs).
// merge.go:41 states the contract -- the newest pair, first in the input,
// wins -- and merge_test.go:25,53 checks it; LSM_TIE_INPUT implements that
// contract: equal keys leave in input order.  LSM_TIE_GOHEAP reproduces the
// heap exactly: the sort below gives dense key ranks, one host thread replays
// heap.Push / heap.Pop over them (a single dependent chain), and the pop
// order replaces the sorted order before steps 3-5.
//
// GPU shape:
//   1. key statistics in one pass (max / min key length; per 8-byte chunk the
//      OR and AND of every key's big-endian chunk), per-block partials reduced
//      on the host, which picks the radix passes;
//   2. LSD radix passes (rocPRIM onesweep, stable) on the key length, then
//      chunk D-1 .. chunk 0 (zero padded), each over only the bits that vary:
//      the result is Go string order with input order on full ties;
//   3. group flags (a key differing from its predecessor starts a group; an
//      empty key is its own group because "" is never deduplicated) and the
//      candidate of each group: its first pair that may be written;
//   4. one scan of the candidates' (size, count) into interleaved sums, then
//      one wave walks the file boundaries -- one probe round per file when it
//      starts a group, and the windows around the next files' predicted ends
//      ride in the same round trip (up to kWalkAhead files per round); a flush inside a group makes the next writable pair of
//      that group a write of its own (the "extra" of the next file);
//   5. emit: each candidate's output slot from its file's start.
// Steps 3-5 are exact for any input; only the tie order is specified above.

#include <rocprim/device/device_radix_sort.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "common.h"

namespace lsm {
namespace {

constexpr uint32_t kMergeThreads = 256;
constexpr uint32_t kStatBlocks = 1024;
constexpr uint32_t kFastChunks = 4;               // chunks counted in the first pass (32 B keys)
constexpr uint32_t kMaxChunks = kKeyCap / 8 + 1;  // 1 MiB keys
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kScanPer = 2;  // 16: lanes 256 B apart (strided stores); A/B compact 1.359 -> 1.348 ms
constexpr uint32_t kScanTile = kMergeThreads * kScanPer;

// Go's kv.DeletedValue, "～DELETED～" (kv/kv.go:29), 13 bytes
__constant__ uint8_t kTomb[13] = {0xEF, 0xBD, 0x9E, 'D', 'E', 'L', 'E', 'T',
                                  'E', 'D', 0xEF, 0xBD, 0x9E};

struct View {
    uint64_t ko, vo;
    uint32_t kl, vl;
};

struct MergeIn {
    const uint8_t *bytes;
    const lsm_rec_desc *kd;
    const lsm_rec_desc *vd;  // null: KV records (value follows the key)
    uint32_t n;
};

__device__ __forceinline__ View view(const MergeIn &m, uint32_t i) {
    const u32x4 k = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(m.kd) + i);
    View v;
    v.ko = ((uint64_t)k.y << 32 | k.x) + 4;
    v.kl = k.z;
    if (m.vd) {
        const u32x4 d = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(m.vd) + i);
        v.vo = ((uint64_t)d.y << 32 | d.x) + 4;
        v.vl = d.w;
    } else {
        v.vo = v.ko + 4 + v.kl;
        v.vl = k.w;
    }
    return v;
}

// Four bytes at any address from the two aligned dwords that cover them
// (inputs are readable to the next 16-byte multiple past their last byte,
// and keys and values sit at rec_off + 4 or later).
__device__ __forceinline__ uint32_t ld_u32_any(const uint8_t *p) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const gptr_t<const uint32_t> q = gbl_at<const uint32_t>(a & ~(uintptr_t)3);
    return funnel(q[0], q[1], (uint32_t)a);
}

// Big-endian 8-byte chunk d of a key of kl bytes at p, zero past its end.
__device__ __forceinline__ uint64_t key_chunk(const uint8_t *p, uint32_t kl, uint32_t d) {
    const uint32_t b0 = 8 * d;
    if (b0 >= kl) return 0;
    const uint64_t c = (uint64_t)bswap32(ld_u32_any(p + b0)) << 32 | bswap32(ld_u32_any(p + b0 + 4));
    const uint32_t have = kl - b0;
    return have >= 8 ? c : c & ~(~0ull >> (8 * have));
}

__device__ __forceinline__ uint64_t wave_or64(uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ uint64_t wave_and64(uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) v &= __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ uint64_t wave_max64(uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t t = __shfl_xor(v, o);
        v = t > v ? t : v;
    }
    return v;
}
__device__ __forceinline__ uint64_t wave_min64(uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t t = __shfl_xor(v, o);
        v = t < v ? t : v;
    }
    return v;
}

// Per-block partial statistics: [0] max key length, [1] min key length,
// [2] OR / [3] AND of the key lengths, then for chunks d < kFastChunks the OR
// and AND of chunk d over keys longer than 8d (shorter keys hold 0 there:
// the host folds that in with the minimum key length).
constexpr uint32_t kStatWords = 4 + 2 * kFastChunks;

__global__ __launch_bounds__(kMergeThreads) void merge_stats_kernel(MergeIn m, uint64_t *part) {
    __shared__ uint64_t red[kMergeThreads / kWave][kStatWords];
    uint64_t s[kStatWords];
    s[0] = 0; s[1] = ~0ull; s[2] = 0; s[3] = ~0ull;
    for (uint32_t d = 0; d < kFastChunks; d++) {
        s[4 + 2 * d] = 0;
        s[5 + 2 * d] = ~0ull;
    }
    for (uint32_t i = blockIdx.x * kMergeThreads + threadIdx.x; i < m.n;
         i += gridDim.x * kMergeThreads) {
        const View v = view(m, i);
        s[0] = v.kl > s[0] ? v.kl : s[0];
        s[1] = v.kl < s[1] ? v.kl : s[1];
        s[2] |= v.kl;
        s[3] &= v.kl;
#pragma unroll
        for (uint32_t d = 0; d < kFastChunks; d++) {
            if (v.kl > 8 * d) {
                const uint64_t c = key_chunk(m.bytes + v.ko, v.kl, d);
                s[4 + 2 * d] |= c;
                s[5 + 2 * d] &= c;
            }
        }
    }
    s[0] = wave_max64(s[0]);
    s[1] = wave_min64(s[1]);
    for (uint32_t t = 2; t < kStatWords; t += 2) {
        s[t] = wave_or64(s[t]);
        s[t + 1] = wave_and64(s[t + 1]);
    }
    const uint32_t w = threadIdx.x / kWave;
    if (lane_id() == 0)
        for (uint32_t t = 0; t < kStatWords; t++) red[w][t] = s[t];
    __syncthreads();
    if (threadIdx.x < kStatWords) {
        const uint32_t t = threadIdx.x;
        uint64_t r = red[0][t];
        for (uint32_t x = 1; x < kMergeThreads / kWave; x++) {
            const uint64_t y = red[x][t];
            if (t == 0) r = y > r ? y : r;
            else if (t == 1) r = y < r ? y : r;
            else if (t & 1) r &= y;
            else r |= y;
        }
        part[(uint64_t)blockIdx.x * kStatWords + t] = r;
    }
}

// Long keys (chunks kFastChunks .. D-1): OR / AND by atomics on orand[2d],
// orand[2d + 1], initialized by the host.
__global__ __launch_bounds__(kMergeThreads) void merge_long_stats_kernel(MergeIn m, uint32_t D,
                                                                         uint64_t *orand) {
    const uint32_t i0 = blockIdx.x * kMergeThreads + threadIdx.x, step = gridDim.x * kMergeThreads;
    for (uint32_t d = kFastChunks; d < D; d++) {
        uint64_t o = 0, a = ~0ull;
        for (uint32_t i = i0; i < m.n; i += step) {
            const View v = view(m, i);
            if (v.kl > 8 * d) {
                const uint64_t c = key_chunk(m.bytes + v.ko, v.kl, d);
                o |= c;
                a &= c;
            }
        }
        o = wave_or64(o);
        a = wave_and64(a);
        if (lane_id() == 0) {
            atomicOr(reinterpret_cast<unsigned long long *>(&orand[2 * d]), (unsigned long long)o);
            atomicAnd(reinterpret_cast<unsigned long long *>(&orand[2 * d + 1]),
                      (unsigned long long)a);
        }
    }
}

// One radix pass sorts a 64-bit key packed from several fields (the key
// length and 8-byte chunks), each reduced to the bits that vary across all
// keys: bits that never vary cannot decide an order, and compressing the
// rest keeps their order (pext), so whole keys of a few varying bytes sort
// in one pass instead of one pass per chunk.
constexpr uint32_t kGroupFields = 8;
struct SortGroup {
    uint32_t nf;
    uint32_t field[kGroupFields];  // chunk index, or kNone for the key length; most significant first
    uint64_t mask[kGroupFields];   // its varying bits
};

// bits of v under mask, packed toward bit 0 in order (mask is wave-uniform)
__device__ __forceinline__ uint64_t pext64(uint64_t v, uint64_t mask) {
    uint64_t r = 0;
    uint32_t pos = 0;
    while (mask) {
        const uint32_t lo = (uint32_t)__builtin_ctzll(mask);
        const uint64_t m = mask >> lo;
        const uint32_t len = ~m ? (uint32_t)__builtin_ctzll(~m) : 64 - lo;
        const uint64_t bits = len >= 64 ? v >> lo : (v >> lo) & ((1ull << len) - 1);
        r |= bits << pos;
        pos += len;
        mask = len + lo >= 64 ? 0 : mask & ~(((1ull << len) - 1) << lo);
    }
    return r;
}

// sort key of sorted position j for one pass (32-bit keys when the pass
// holds at most 32 varying bits: a third less traffic per radix pass)
template <class K>
__global__ __launch_bounds__(kMergeThreads) void merge_extract_kernel(MergeIn m, const uint32_t *perm,
                                                                      SortGroup g, K *keys) {
    const uint32_t j = blockIdx.x * kMergeThreads + threadIdx.x;
    if (j >= m.n) return;
    const uint32_t i = perm ? perm[j] : j;
    const View v = view(m, i);
    uint64_t key = 0;
    for (uint32_t t = 0; t < g.nf; t++) {
        const uint64_t x = g.field[t] == kNone ? v.kl : key_chunk(m.bytes + v.ko, v.kl, g.field[t]);
        const uint32_t bits = (uint32_t)__builtin_popcountll(g.mask[t]);
        key = (bits >= 64 ? 0 : key << bits) | pext64(x, g.mask[t]);
    }
    keys[j] = (K)key;
}

__global__ __launch_bounds__(kMergeThreads) void merge_iota_kernel(uint32_t *perm, uint32_t n) {
    const uint32_t j = blockIdx.x * kMergeThreads + threadIdx.x;
    if (j < n) perm[j] = j;
}

__device__ __forceinline__ bool keys_equal(const uint8_t *b, const View &x, const View &y) {
    if (x.kl != y.kl) return false;
    for (uint32_t d = 0; 8 * d < x.kl; d++)
        if (key_chunk(b + x.ko, x.kl, d) != key_chunk(b + y.ko, y.kl, d)) return false;
    return true;
}

__device__ __forceinline__ bool is_tombstone(const uint8_t *b, const View &v) {
    if (v.vl != 13) return false;
    const uint8_t *p = b + v.vo;
    // "～DELETED～" as little-endian dwords of bytes 0-3, 4-7, 8-11, then byte 12
    return ld_u32_any(p) == 0x449EBDEFu && ld_u32_any(p + 4) == 0x54454C45u &&
           ld_u32_any(p + 8) == 0xBDEF4445u && p[12] == kTomb[12];
}

// flags[j]: bit 0 = starts a group, bit 1 = may be written (not a tombstone
// dropped at level 6); csize[j] = the pair's EstimateSize (16 + key + value,
// kv.go:118-121), which merge_candidate_kernel keeps or zeroes in place (the
// view is loaded here anyway: no second gather through perm)
__global__ __launch_bounds__(kMergeThreads) void merge_flags_kernel(MergeIn m, const uint32_t *perm,
                                                                    int level, uint8_t *flags,
                                                                    uint32_t *csize) {
    const uint32_t j = blockIdx.x * kMergeThreads + threadIdx.x;
    if (j >= m.n) return;
    const View v = view(m, perm[j]);
    bool gs = j == 0 || v.kl == 0;
    if (!gs) gs = !keys_equal(m.bytes, v, view(m, perm[j - 1]));
    const bool wr = level < 6 || !is_tombstone(m.bytes, v);
    flags[j] = (uint8_t)((gs ? 1 : 0) | (wr ? 2 : 0));
    csize[j] = 16 + v.kl + v.vl;
}

// eq[j] = 1 when sorted position j holds the same key as j - 1 (plain key
// equality: for container/heap "" equals "", merge.go:21-23's Less is key <)
__global__ __launch_bounds__(kMergeThreads) void merge_eq_kernel(MergeIn m, const uint32_t *perm,
                                                                 uint8_t *eq) {
    const uint32_t j = blockIdx.x * kMergeThreads + threadIdx.x;
    if (j >= m.n) return;
    eq[j] = j > 0 && keys_equal(m.bytes, view(m, perm[j]), view(m, perm[j - 1]));
}

// candidate = the first pair of its group that may be written; the backward
// scan stops at the first writable pair or the group start, so each run of
// dropped tombstones is scanned by one pair only (O(n) in total).
// csize[j] = EstimateSize of a candidate (kv.go:118-121, >= 16), else 0.
__global__ __launch_bounds__(kMergeThreads) void merge_candidate_kernel(MergeIn m,
                                                                        const uint8_t *flags,
                                                                        uint32_t *csize) {
    const uint32_t j = blockIdx.x * kMergeThreads + threadIdx.x;
    if (j >= m.n) return;
    const uint8_t f = flags[j];
    bool c = (f & 2) != 0;
    if (c && !(f & 1)) {
        for (uint32_t k = j; k-- > 0;) {
            const uint8_t g = flags[k];
            if (g & 2) { c = false; break; }
            if (g & 1) break;
        }
    }
    if (!c) csize[j] = 0;  // candidates keep the size merge_flags_kernel wrote
}

// ---- interleaved exclusive sums of candidate sizes and counts -----------

struct SumPair {
    uint64_t s, c;  // bytes and candidates before position j
};

__device__ __forceinline__ SumPair block_excl_scan2(uint64_t s, uint64_t c, SumPair *total) {
    __shared__ uint64_t ws_[kMergeThreads / kWave], wc_[kMergeThreads / kWave];
    uint64_t ts, tc;
    const uint64_t xs = wave_excl_scan64(s, &ts), xc = wave_excl_scan64(c, &tc);
    const uint32_t w = threadIdx.x / kWave;
    if (lane_id() == 0) {
        ws_[w] = ts;
        wc_[w] = tc;
    }
    __syncthreads();
    uint64_t ps = 0, pc = 0, as = 0, ac = 0;
    for (uint32_t i = 0; i < kMergeThreads / kWave; i++) {
        if (i < w) {
            ps += ws_[i];
            pc += wc_[i];
        }
        as += ws_[i];
        ac += wc_[i];
    }
    __syncthreads();
    *total = SumPair{as, ac};
    return SumPair{xs + ps, xc + pc};
}

__global__ __launch_bounds__(kMergeThreads) void merge_scan_tiles(const uint32_t *csize, uint32_t n,
                                                                  SumPair *part) {
    uint64_t s = 0, c = 0;
    const uint64_t i0 = (uint64_t)blockIdx.x * kScanTile + threadIdx.x * kScanPer;
    for (uint32_t t = 0; t < kScanPer; t++) {
        const uint32_t v = i0 + t < n ? csize[i0 + t] : 0;
        s += v;
        c += v != 0;
    }
    SumPair tot;
    block_excl_scan2(s, c, &tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kMergeThreads) void merge_scan_partials(SumPair *part, uint32_t ntiles,
                                                                     SumPair *sc, uint32_t n) {
    SumPair carry{0, 0};
    for (uint32_t t0 = 0; t0 < ntiles; t0 += kMergeThreads) {
        const uint32_t t = t0 + threadIdx.x;
        const SumPair v = t < ntiles ? part[t] : SumPair{0, 0};
        SumPair tot;
        const SumPair x = block_excl_scan2(v.s, v.c, &tot);
        if (t < ntiles) part[t] = SumPair{carry.s + x.s, carry.c + x.c};
        carry.s += tot.s;
        carry.c += tot.c;
    }
    if (threadIdx.x == 0) sc[n] = carry;
}

__global__ __launch_bounds__(kMergeThreads) void merge_scan_apply(const uint32_t *csize, uint32_t n,
                                                                  const SumPair *part, SumPair *sc) {
    uint32_t v[kScanPer];
    uint64_t s = 0, c = 0;
    const uint64_t i0 = (uint64_t)blockIdx.x * kScanTile + threadIdx.x * kScanPer;
    for (uint32_t t = 0; t < kScanPer; t++) {
        v[t] = i0 + t < n ? csize[i0 + t] : 0;
        s += v[t];
        c += v[t] != 0;
    }
    SumPair tot;
    const SumPair x = block_excl_scan2(s, c, &tot);
    uint64_t ps = x.s + part[blockIdx.x].s, pc = x.c + part[blockIdx.x].c;
    for (uint32_t t = 0; t < kScanPer; t++) {
        if (i0 + t < n) sc[i0 + t] = SumPair{ps, pc};
        ps += v[t];
        pc += v[t] != 0;
    }
}

// ---- the file walk --------------------------------------------------------

struct MergeFile {
    uint32_t p;      // first sorted position of the file
    uint32_t extra;  // sorted position of the group continuation written first, or kNone
    uint64_t o;      // first output slot
};

struct WalkArgs {
    MergeIn m;
    const uint32_t *perm;
    const uint8_t *flags;
    const SumPair *sc;  // n + 1
    uint64_t threshold;
    MergeFile *files;
    uint32_t *out;
    uint64_t *counts;   // [0] = written pairs, [1] = files, [2] = most pairs in one file
};

// smallest k in [lo, hi] with sc[k].s >= t, given sc[hi].s >= t
__device__ uint32_t wave_lower_bound(const SumPair *sc, uint32_t lo, uint32_t hi, uint64_t t) {
    const uint32_t lane = lane_id();
    while (hi > lo) {
        // lane l probes lo + l*step, the last lane probes hi (>= t), so the
        // first lane at or above t exists and the lane before it is below
        const uint32_t span = hi - lo;
        const uint32_t step = span >= 63 ? (span + 62) / 63 : 1;
        uint32_t k = lo + lane * step;
        if (k > hi || lane == kWave - 1) k = hi;
        const uint64_t ge = __ballot(sc[k].s >= t);
        const uint32_t f = (uint32_t)__builtin_ctzll(ge);
        if (f == 0) return uni(lo);
        uint32_t kf = lo + f * step;
        if (kf > hi || f == kWave - 1) kf = hi;
        lo = uni(lo + (f - 1) * step + 1);
        hi = uni(kf);
    }
    return uni(lo);
}

// One wave walks the files (merge.go:57-91): file f starts at sorted position
// p; if p continues a group whose pair was written just before the flush,
// lastWrittenKey is "" again and the group's next writable pair is written
// (the file's "extra"); then come the candidates of later groups until the
// size reaches the threshold.  The common case -- p starts a group and the
// file spans about as many positions as the last one -- takes one round of
// loads: lane 0 reads flags[p] and sc[p] while lanes 1..63 probe sc around
// the predicted end.
constexpr uint32_t kWalkAhead = 8;  // windows (files) per round trip of the walk

__device__ __forceinline__ uint64_t lane_u64(uint64_t v, uint32_t l) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), l) << 32 |
           (uint32_t)__builtin_amdgcn_readlane((uint32_t)v, l);
}

__global__ __launch_bounds__(64) void merge_walk_kernel(WalkArgs a) {
    const uint32_t n = a.m.n, lane = lane_id();
    const SumPair tail = a.sc[n];
    uint32_t p = 0, nf = 0, span = 0;
    uint64_t o = 0, most = 0;
    while (p < n) {
        // speculative round: lane 0 reads flags[p] and sc[p]; every lane reads
        // sc at four positions of the window [w0, w0 + 256) around the
        // predicted end (all five loads in one round trip)
        const uint32_t w0 = span > 128 ? p + span - 127 : p + 1;
        SumPair q[4];
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) {
            const uint32_t k = w0 + lane + kWave * i;
            q[i] = a.sc[k <= n ? k : n];
        }
        // ... and, in the same round trip, the windows around the next
        // kWalkAhead - 1 predicted ends and the flags of every window: files
        // that start a group chain through them without another round
        const bool ahead = span > 128;
        const uint32_t span0 = span;
        SumPair qx[kWalkAhead - 1][4];
        uint8_t fx[kWalkAhead][4];
#pragma unroll
        for (uint32_t j = 0; j < kWalkAhead; j++) {
#pragma unroll
            for (uint32_t i = 0; i < 4; i++) {
                const uint64_t k = (uint64_t)w0 + (uint64_t)j * span0 + lane + kWave * i;
                const uint32_t kc = k <= n ? (uint32_t)k : n;
                if (j) qx[j - 1][i] = a.sc[kc];  // unconditional: no branch per load
                fx[j][i] = a.flags[kc < n ? kc : n - 1];
            }
        }
        const SumPair q0 = a.sc[p];
        const uint8_t fl0 = lane == 0 ? a.flags[p] : 0;
        const bool starts = p == 0 || (__builtin_amdgcn_readfirstlane(fl0) & 1);
        const uint64_t S0 = uni64(q0.s), C0 = uni64(q0.c);
        uint32_t g = p, w = kNone, e = kNone;
        uint64_t wsize = 0, Cg = C0;
        bool done = false, have_ce = false;
        uint64_t Ce = 0, Sk = 0;  // at the end found in window 0
        uint32_t fk = 0;
        if (starts) {
            const uint64_t t = S0 + a.threshold;
            if (tail.s < t) {
                done = true;  // the rest fits in this file
            } else {
#pragma unroll
                for (uint32_t i = 0; i < 4; i++) {
                    const uint64_t ge = __ballot(q[i].s >= t);
                    if (!ge) continue;
                    const uint32_t f = (uint32_t)__builtin_ctzll(ge);
                    const uint32_t k = w0 + kWave * i + f;  // first probe at or above t
                    if (k > w0 || k == p + 1) {  // the position before k is below t
                        e = k - 1;
                        done = true;
                        Ce = lane_u64(q[i].c, f);
                        Sk = lane_u64(q[i].s, f);
                        fk = (uint32_t)__builtin_amdgcn_readlane((uint32_t)fx[0][i], f);
                        have_ce = true;
                    }
                    break;
                }
            }
        } else {
            // the rest of the group: its end and its first writable pair
            for (uint32_t q0 = p;; q0 += kWave) {
                const uint32_t qq = q0 + lane;
                const uint8_t f = qq < n ? a.flags[qq] : 1;
                const bool end = qq >= n || (qq > p && (f & 1));
                const uint64_t em = __ballot(end);
                const uint64_t wm = __ballot(!end && (f & 2)) & (em ? (em & -em) - 1 : ~0ull);
                if (w == kNone && wm) w = uni(q0 + (uint32_t)__builtin_ctzll(wm));
                if (em) {
                    g = uni(q0 + (uint32_t)__builtin_ctzll(em));
                    break;
                }
            }
            if (w != kNone) {
                const View v = view(a.m, a.perm[w]);
                wsize = 16 + (uint64_t)v.kl + v.vl;
            }
            Cg = g < n ? uni64(a.sc[g].c) : tail.c;
            if (w != kNone && wsize >= a.threshold) {
                e = w;
                done = true;
            }
        }
        if (!done) {
            const uint64_t Sg = g < n ? uni64(a.sc[g].s) : tail.s;
            const uint64_t t = Sg + (a.threshold - wsize);
            if (tail.s >= t) e = wave_lower_bound(a.sc, g + 1, n, t) - 1;
        }
        const uint32_t end = e == kNone ? n : e + 1;
        if (!have_ce) Ce = end < n ? uni64(a.sc[end].c) : tail.c;
        const uint64_t nw = (w != kNone ? 1 : 0) + (end > g ? Ce - Cg : 0);
        if (nw == 0) break;  // nothing left to write: no file (builder.size == 0)
        if (lane == 0) {
            a.files[nf] = MergeFile{p, w, o};
            if (w != kNone) a.out[o] = a.perm[w];
        }
        o += nw;
        most = nw > most ? nw : most;
        nf++;
        span = end - g;
        p = end;
        if (!(starts && have_ce && ahead)) continue;
        // chain: file j starts at p (found in window j - 1, with its S, C and
        // flags); its end is exact when it lies inside window j
        uint64_t Sj = Sk, Cj = Ce;
        uint32_t fj = fk;
#pragma unroll
        for (uint32_t j = 1; j < kWalkAhead; j++) {
            if (p >= n || !(fj & 1)) break;  // done, or a group continues: general round
            const uint64_t t = Sj + a.threshold;
            if (tail.s < t) break;  // the last file: general round
            const uint64_t wj = (uint64_t)w0 + (uint64_t)j * span0;
            bool hit = false;
            uint32_t k = 0, fn = 0;
            uint64_t Cn = 0, Sn = 0;
#pragma unroll
            for (uint32_t i = 0; i < 4; i++) {
                const uint64_t ge = __ballot(qx[j - 1][i].s >= t);
                if (!ge) continue;
                const uint32_t f = (uint32_t)__builtin_ctzll(ge);
                const uint64_t kk = wj + kWave * i + f;
                hit = kk > wj || kk == (uint64_t)p + 1;  // the position before is below t
                k = (uint32_t)kk;
                Cn = lane_u64(qx[j - 1][i].c, f);
                Sn = lane_u64(qx[j - 1][i].s, f);
                fn = (uint32_t)__builtin_amdgcn_readlane((uint32_t)fx[j][i], f);
                break;
            }
            if (!hit || Cn == Cj) break;
            if (lane == 0) a.files[nf] = MergeFile{p, kNone, o};
            o += Cn - Cj;
            most = Cn - Cj > most ? Cn - Cj : most;
            nf++;
            span = k - p;
            p = k;
            Cj = Cn;
            Sj = Sn;
            fj = fn;
        }
    }
    if (lane == 0) {
        a.files[nf] = MergeFile{n, kNone, o};
        a.counts[0] = o;
        a.counts[1] = nf;
        a.counts[2] = most;
    }
}

// each candidate's output slot: its file's first slot, after the extra, plus
// the candidates before it in the file
__global__ __launch_bounds__(kMergeThreads) void merge_emit_kernel(
    const uint32_t *perm, const SumPair *sc, const uint32_t *csize, const MergeFile *files,
    const uint64_t *counts, uint32_t n, uint32_t *out, uint64_t *file_start) {
    __shared__ uint32_t s_lo;
    const uint32_t j0 = blockIdx.x * kMergeThreads, j = j0 + threadIdx.x;
    const uint32_t nf = (uint32_t)counts[1];
    if (j <= nf && file_start) file_start[j] = files[j].o;
    // the file of the workgroup's first position: one search per workgroup;
    // a position's file is then at most a few files further (a file spans
    // about threshold / pair size positions), else searched again
    auto last_le = [&](uint32_t lo, uint32_t hi, uint32_t x) {  // last file in [lo, hi) with p <= x
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) / 2;
            if (files[mid].p <= x) lo = mid; else hi = mid;
        }
        return lo;
    };
    if (threadIdx.x == 0) s_lo = nf ? last_le(0, nf, j0) : 0;
    __syncthreads();
    if (j >= n || !csize[j]) return;
    uint32_t lo = s_lo;
    for (uint32_t step = 0; lo + 1 < nf && files[lo + 1].p <= j; step++) {
        if (step == 4) { lo = last_le(lo, nf, j); break; }
        lo++;
    }
    if (nf == 0 || files[lo].p > j || j >= files[lo + 1].p) return;  // past the last file
    const MergeFile F = files[lo];
    out[F.o + (F.extra != kNone ? 1 : 0) + (sc[j].c - sc[F.p].c)] = perm[j];
}

// ---- gather: the written pairs -> a CSR record batch (build input) --------

__global__ __launch_bounds__(kMergeThreads) void gather_lens_kernel(MergeIn m, const uint32_t *idx,
                                                                    uint32_t nout, uint32_t *klen,
                                                                    uint32_t *vlen) {
    const uint32_t j = blockIdx.x * kMergeThreads + threadIdx.x;
    if (j >= nout) return;
    const View v = view(m, idx[j]);
    klen[j] = v.kl;
    vlen[j] = v.vl;
}

// One wave per 64 pairs.  Their keys form one contiguous output range and
// their values another; both are cut into 16-byte chunks (aligned in the
// output) numbered in one space, keys first:
//   1. each lane marks, in an LDS map, the chunks that start inside its key
//      or its value;
//   2. lanes take four chunks at a time and issue every source load before
//      any store (a round trip covers four chunks): a chunk inside one
//      key or value is five aligned source dwords funnel-shifted into one
//      16-byte store; any other chunk (it straddles pairs or an end of the
//      range) is queued;
//   3. the queue is drained four lanes per chunk, a dword (or its bytes) each.
// Chunks are handled kMapChunks at a time (any pair size).
constexpr uint32_t kMapChunks = 1024;
constexpr uint32_t kUnroll = 4;

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(kMergeThreads) void gather_copy_kernel(
    MergeIn m, const uint32_t *idx, uint32_t nout, const uint64_t *koff, const uint64_t *voff,
    uint8_t *keys, uint8_t *vals) {
    constexpr uint32_t W = kMergeThreads / kWave;
    __shared__ uint64_t s_dst[W][2][kWave + 1];
    __shared__ uint64_t s_src[W][2][kWave];
    __shared__ uint8_t s_map[W][kMapChunks];
    __shared__ uint16_t s_q[W][kMapChunks];
    const uint32_t w = threadIdx.x / kWave, lane = lane_id();
    const uint32_t j0 = (blockIdx.x * W + w) * kWave;
    if (j0 >= nout) return;
    const uint32_t cnt = nout - j0 < kWave ? nout - j0 : kWave;
    uint64_t d0[2] = {0, 0}, d1[2] = {0, 0};
    if (lane < cnt) {
        const View v = view(m, idx[j0 + lane]);
        d0[0] = koff[j0 + lane];
        d0[1] = voff[j0 + lane];
        d1[0] = d0[0] + v.kl;
        d1[1] = d0[1] + v.vl;
        s_src[w][0][lane] = v.ko;
        s_src[w][1][lane] = v.vo;
        s_dst[w][0][lane] = d0[0];
        s_dst[w][1][lane] = d0[1];
    }
    if (lane == 0) {
        s_dst[w][0][cnt] = koff[j0 + cnt];
        s_dst[w][1][cnt] = voff[j0 + cnt];
    }
    wave_sync();
    uint64_t A[2], B[2], X[2];
    uint32_t nc[2];
    for (int h = 0; h < 2; h++) {
        A[h] = s_dst[w][h][0];
        B[h] = s_dst[w][h][cnt];
        X[h] = A[h] & ~(uint64_t)15;
        nc[h] = B[h] > A[h] ? (uint32_t)((B[h] - X[h] + 15) / 16) : 0;
    }
    if (!vals) nc[1] = 0;  // keys only (lsm_build_sst_views reads the values in place)
    const gptr_t<uint8_t> dsts[2] = {gbl(keys), gbl(vals)};
    const gptr_t<const uint8_t> src = gbl(m.bytes);
    const uint32_t total = nc[0] + nc[1];
    for (uint32_t P = 0; P < total; P += kMapChunks) {
        const uint32_t np = total - P < kMapChunks ? total - P : kMapChunks;
        // 1. chunks whose first byte lies in my key / value
        for (int h = 0; h < 2; h++) {
            if (lane < cnt && d1[h] > d0[h] && d1[h] - 1 >= X[h]) {
                const uint64_t lo = d0[h] > X[h] ? (d0[h] - X[h] + 15) / 16 : 0;
                const uint64_t hi = (d1[h] - 1 - X[h]) / 16;
                const uint64_t base = h ? nc[0] : 0;
                const uint64_t c_lo = base + lo > P ? base + lo : P;
                const uint64_t c_hi = base + hi < (uint64_t)P + np - 1 ? base + hi : (uint64_t)P + np - 1;
                for (uint64_t c = c_lo; c <= c_hi; c++) s_map[w][c - P] = (uint8_t)lane;
            }
        }
        wave_sync();
        // 2. chunks inside one key / value, four per lane per round; queue the rest
        uint32_t qn = 0;
        for (uint32_t c0 = 0; c0 < np; c0 += kUnroll * kWave) {
            uint32_t q[kUnroll][5];
            uint32_t sh[kUnroll];
            gptr_t<uint8_t> out[kUnroll];
            bool reg[kUnroll];
#pragma unroll
            for (uint32_t u = 0; u < kUnroll; u++) {
                const uint32_t c = c0 + u * kWave + lane;
                reg[u] = false;
                out[u] = nullptr;
                sh[u] = 0;
                if (c < np) {
                    const uint32_t cid = P + c;
                    const int h = cid >= nc[0];
                    const uint64_t x = X[h] + 16 * (uint64_t)(cid - (h ? nc[0] : 0));
                    if (x >= A[h] && x + 16 <= B[h]) {
                        const uint32_t r = s_map[w][c];
                        const uint64_t e0 = s_dst[w][h][r], e1 = s_dst[w][h][r + 1];
                        if (x + 16 <= e1) {
                            reg[u] = true;
                            const uintptr_t sa =
                                reinterpret_cast<uintptr_t>(m.bytes + s_src[w][h][r] + (x - e0));
                            const gptr_t<const uint32_t> qa = gbl_at<const uint32_t>(sa & ~(uintptr_t)3);
                            sh[u] = (uint32_t)sa;
                            out[u] = dsts[h] + x;
#pragma unroll
                            for (int t = 0; t < 5; t++) q[u][t] = qa[t];
                        }
                    }
                }
            }
#pragma unroll
            for (uint32_t u = 0; u < kUnroll; u++) {
                if (reg[u]) {
                    u32x4 o;
                    o.x = funnel(q[u][0], q[u][1], sh[u]);
                    o.y = funnel(q[u][1], q[u][2], sh[u]);
                    o.z = funnel(q[u][2], q[u][3], sh[u]);
                    o.w = funnel(q[u][3], q[u][4], sh[u]);
                    *(gptr_t<u32x4>)out[u] = o;
                }
                const uint32_t c = c0 + u * kWave + lane;
                const bool irr = c < np && !reg[u];
                const uint64_t im = __ballot(irr);
                if (irr) s_q[w][qn + mbcnt(im)] = (uint16_t)c;
                qn += (uint32_t)__builtin_popcountll(im);
            }
        }
        wave_sync();
        // 3. queued chunks, four lanes (one dword each) per chunk
        for (uint32_t i0 = 0; i0 < qn; i0 += kWave / 4) {
            const uint32_t i = i0 + lane / 4;
            if (i >= qn) continue;
            const uint32_t c = s_q[w][i], cid = P + c;
            const int h = cid >= nc[0];
            const uint64_t x = X[h] + 16 * (uint64_t)(cid - (h ? nc[0] : 0));
            const uint64_t xd = x + 4 * (lane & 3);
            if (xd >= B[h]) continue;
            uint32_t r = x >= A[h] ? s_map[w][c] : 0;
            const uint64_t *sd = s_dst[w][h];
            const uint64_t *ss = s_src[w][h];
            const gptr_t<uint8_t> dst = dsts[h];
            while (r + 1 < cnt && xd >= sd[r + 1]) r++;
            if (xd >= A[h] && xd + 4 <= B[h] && xd >= sd[r] && xd + 4 <= sd[r + 1]) {
                *(gptr_t<uint32_t>)(dst + xd) = ld_u32_any(m.bytes + ss[r] + (xd - sd[r]));
            } else {
                for (uint32_t u = 0; u < 4; u++) {
                    const uint64_t b = xd + u;
                    if (b < A[h] || b >= B[h]) continue;
                    while (b >= sd[r + 1]) r++;
                    dst[b] = src[ss[r] + (b - sd[r])];
                }
            }
        }
        wave_sync();
    }
}

// ---- .sst image sizes of the files a merge produced ----------------------

__global__ __launch_bounds__(kMergeThreads) void sst_sizes_kernel(const uint64_t *koff,
                                                                  const uint64_t *voff,
                                                                  const uint64_t *file_start,
                                                                  uint32_t nfile, uint64_t filter,
                                                                  uint64_t *size) {
    const uint32_t f = blockIdx.x * kMergeThreads + threadIdx.x;
    if (f >= nfile) return;
    const uint64_t r0 = file_start[f], r1 = file_start[f + 1];
    uint64_t hdr = 8;
    if (r1 > r0) hdr += (koff[r0 + 1] - koff[r0]) + (koff[r1] - koff[r1 - 1]);
    const uint64_t nr = r1 - r0;
    // Header | Filter | V region (4 + vlen) | IDX region (4 + klen + 8) | Footer
    size[f] = hdr + filter + 4 * nr + (voff[r1] - voff[r0]) + 12 * nr + (koff[r1] - koff[r0]) + 32;
}

// The images' layout on the device: each file's size (as sst_sizes_kernel)
// and its offset in one output buffer, sizes rounded up to `align`;
// file_off[nfile] = the total.  One workgroup (a few thousand files at most
// per compaction), tile after tile with a carry.
__global__ __launch_bounds__(kMergeThreads) void sst_layout_kernel(const uint64_t *koff,
                                                                   const uint64_t *voff,
                                                                   const uint64_t *file_start,
                                                                   uint32_t nfile, uint64_t filter,
                                                                   uint64_t align, uint64_t *size,
                                                                   uint64_t *file_off) {
    uint64_t carry = 0;
    for (uint32_t f0 = 0; f0 < nfile; f0 += kMergeThreads) {
        const uint32_t f = f0 + threadIdx.x;
        uint64_t sz = 0;
        if (f < nfile) {
            const uint64_t r0 = file_start[f], r1 = file_start[f + 1], nr = r1 - r0;
            uint64_t hdr = 8;
            if (r1 > r0) hdr += (koff[r0 + 1] - koff[r0]) + (koff[r1] - koff[r1 - 1]);
            sz = hdr + filter + 4 * nr + (voff[r1] - voff[r0]) + 12 * nr + (koff[r1] - koff[r0]) + 32;
            size[f] = sz;
        }
        SumPair tot;
        const SumPair x = block_excl_scan2((sz + align - 1) / align * align, 0, &tot);
        if (f < nfile) file_off[f] = carry + x.s;
        carry += tot.s;
    }
    if (threadIdx.x == 0) file_off[nfile] = carry;
}

// ---- positional join of decoded .sst files (loadLevelData) ----------------

__device__ __forceinline__ uint64_t sst_pair_count(const lsm_sst_meta &m) {
    // GetKeyValuePairs (sstable.go:248-268): nothing from a failed decode or
    // from a table with no data or no index entries
    return (m.stage == LSM_SST_OK && m.nidx && m.ndata) ? m.nidx : 0;
}

__global__ __launch_bounds__(kMergeThreads) void sst_pairs_scan_kernel(const lsm_sst_meta *meta,
                                                                       uint32_t nfile,
                                                                       uint64_t *prefix) {
    uint64_t carry = 0;
    for (uint32_t f0 = 0; f0 < nfile; f0 += kMergeThreads) {
        const uint32_t f = f0 + threadIdx.x;
        const uint64_t c = f < nfile ? sst_pair_count(meta[f]) : 0;
        SumPair tot;
        const SumPair x = block_excl_scan2(c, 0, &tot);
        if (f < nfile) prefix[f] = carry + x.s;
        carry += tot.s;
    }
    if (threadIdx.x == 0) prefix[nfile] = carry;
}

__global__ __launch_bounds__(kMergeThreads) void sst_pairs_copy_kernel(
    const lsm_sst_meta *meta, const uint64_t *file_off, const u32x4 *idx_desc,
    const u32x4 *data_desc, const uint64_t *prefix, u32x4 *key_out, u32x4 *val_out) {
    const uint32_t f = blockIdx.y;
    const uint64_t c = sst_pair_count(meta[f]);
    const uint64_t src = file_off[f] / 4, dst = prefix[f];  // lsm_decode_sst's offset addressing
    for (uint64_t i = (uint64_t)blockIdx.x * kMergeThreads + threadIdx.x; i < c;
         i += (uint64_t)gridDim.x * kMergeThreads) {
        key_out[dst + i] = __builtin_nontemporal_load(&idx_desc[src + i]);
        val_out[dst + i] = __builtin_nontemporal_load(&data_desc[src + i]);
    }
}

// ---- workspace ------------------------------------------------------------

struct MergeWs {
    uint32_t *perm[2];
    uint64_t *keys[2];
    uint8_t *flags;
    uint32_t *csize;
    SumPair *sc;
    SumPair *scan_part;
    MergeFile *files;
    uint64_t *stats;  // [0..1] counts, then the long-key OR/AND words
    uint64_t *part;   // kStatBlocks * kStatWords
    void *sort_tmp;
    size_t sort_bytes;
    size_t total;
};

size_t sort_tmp_bytes(uint32_t n) {
    size_t b = 0, b32 = 0;
    (void)rocprim::radix_sort_pairs(nullptr, b, (uint64_t *)nullptr, (uint64_t *)nullptr,
                                    (uint32_t *)nullptr, (uint32_t *)nullptr, n, 0, 64);
    (void)rocprim::radix_sort_pairs(nullptr, b32, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                    (uint32_t *)nullptr, (uint32_t *)nullptr, n, 0, 32);
    return b > b32 ? b : b32;
}

MergeWs merge_ws_layout(uint8_t *base, uint32_t n) {
    MergeWs w{};
    size_t at = 0;
    auto take = [&](size_t bytes) -> uint8_t * {
        uint8_t *p = base ? base + at : nullptr;
        at += (bytes + 255) & ~(size_t)255;
        return p;
    };
    const size_t nn = n ? n : 1;
    const size_t ntiles = (nn + kScanTile - 1) / kScanTile;
    w.perm[0] = reinterpret_cast<uint32_t *>(take(4 * nn));
    w.perm[1] = reinterpret_cast<uint32_t *>(take(4 * nn));
    w.keys[0] = reinterpret_cast<uint64_t *>(take(8 * nn));
    w.keys[1] = reinterpret_cast<uint64_t *>(take(8 * nn));
    w.flags = take(nn);
    w.csize = reinterpret_cast<uint32_t *>(take(4 * nn));
    w.sc = reinterpret_cast<SumPair *>(take(sizeof(SumPair) * (nn + 1)));
    w.scan_part = reinterpret_cast<SumPair *>(take(sizeof(SumPair) * ntiles));
    w.files = reinterpret_cast<MergeFile *>(take(sizeof(MergeFile) * (nn + 2)));
    w.stats = reinterpret_cast<uint64_t *>(take(8 * (2 + 2 * (size_t)kMaxChunks)));
    w.part = reinterpret_cast<uint64_t *>(take(8 * (size_t)kStatBlocks * kStatWords));
    w.sort_bytes = sort_tmp_bytes(n);
    w.sort_tmp = take(w.sort_bytes);
    w.total = at;
    return w;
}

uint32_t grid_for(uint64_t n) { return (uint32_t)((n + kMergeThreads - 1) / kMergeThreads); }

}  // namespace

// container/heap's pop order (Go heap.go) over dense key ranks: heap.Push of
// pairs 0 .. n-1 (append + up), then heap.Pop until empty (swap(0, n-1),
// down(0, n-1), take the last), with Less(i, j) = rank[i] < rank[j] -- the
// order merge.go:47-66 pops in, equal keys included.  Entries carry
// rank << 32 | index, so one load serves the compare and the move.  One host
// thread: the heap's history is one dependent chain.
void goheap_pop_order(const uint32_t *rank, uint32_t n, uint32_t *order) {
    std::vector<uint64_t> h(n ? n : 1);
    for (uint32_t i = 0; i < n; i++) {  // Push: append, up(h, i)
        const uint64_t x = (uint64_t)rank[i] << 32 | i;
        uint32_t j = i;
        while (j > 0) {
            const uint32_t p = (j - 1) / 2;
            if (!((x >> 32) < (h[p] >> 32))) break;
            h[j] = h[p];
            j = p;
        }
        h[j] = x;
    }
    for (uint32_t r = n; r > 0; r--) {  // Pop: swap(0, r-1), down(0, r-1)
        const uint64_t top = h[0], x = h[r - 1];
        const uint32_t m = r - 1;
        uint32_t i = 0;
        for (;;) {
            const uint32_t j1 = 2 * i + 1;
            if (j1 >= m) break;
            __builtin_prefetch(&h[4 * (uint64_t)i + 3]);  // the grandchildren's line
            uint32_t j = j1;
            if (j1 + 1 < m && (h[j1 + 1] >> 32) < (h[j1] >> 32)) j = j1 + 1;
            if (!((h[j] >> 32) < (x >> 32))) break;
            h[i] = h[j];
            i = j;
        }
        if (m) h[i] = x;
        h[m] = top;
        order[n - r] = (uint32_t)top;
    }
}

}  // namespace lsm

using namespace lsm;

extern "C" int lsm_goheap_pop_order_host(const uint32_t *rank, uint64_t n, uint32_t *order) {
    if (n >= 0xFFFFFFFFull || (n && (!rank || !order))) return LSM_EINVAL;
    goheap_pop_order(rank, (uint32_t)n, order);
    return 0;
}

static_assert(sizeof(MergeFile) == 16, "MergeFile layout");
static_assert(sizeof(SumPair) == 16, "SumPair layout");

extern "C" size_t lsm_merge_kvs_workspace_bytes(uint64_t n) {
    if (n >= 0xFFFFFFFFull) return 0;
    return merge_ws_layout(nullptr, (uint32_t)n).total;
}

extern "C" int lsm_merge_kvs_tie(lsm_ctx *ctx, const uint8_t *d_bytes,
                                 const lsm_rec_desc *d_key_desc, const lsm_rec_desc *d_val_desc,
                                 uint64_t n, int level, uint64_t threshold, int tie,
                                 uint32_t *d_out, uint64_t *d_file_start, uint64_t *h_counts,
                                 void *d_ws, size_t ws_bytes, void *stream) {
    if (!ctx || !h_counts || threshold == 0 || n >= 0xFFFFFFFFull) return LSM_EINVAL;
    if (tie != LSM_TIE_INPUT && tie != LSM_TIE_GOHEAP) return LSM_EINVAL;
    if (n && (!d_bytes || !d_key_desc || !d_out || !d_ws)) return LSM_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    h_counts[0] = h_counts[1] = h_counts[2] = 0;
    if (n == 0) {
        if (d_file_start) LSM_HIP_CHECK(hipMemsetAsync(d_file_start, 0, 8, s));
        return 0;
    }
    const uint32_t N = (uint32_t)n;
    MergeWs w = merge_ws_layout(static_cast<uint8_t *>(d_ws), N);
    if (ws_bytes < w.total) return LSM_ESPACE;
    const MergeIn m{d_bytes, d_key_desc, d_val_desc, N};
    const uint32_t sb = grid_for(n) < kStatBlocks ? grid_for(n) : kStatBlocks;

    // 1. key statistics: one pass, per-block partials reduced here
    hipLaunchKernelGGL(merge_stats_kernel, dim3(sb), dim3(kMergeThreads), 0, s, m, w.part);
    std::vector<uint64_t> part((size_t)sb * kStatWords);
    LSM_HIP_CHECK(hipMemcpyAsync(part.data(), w.part, part.size() * 8, hipMemcpyDeviceToHost, s));
    LSM_HIP_CHECK(hipStreamSynchronize(s));
    uint64_t st[kStatWords];
    for (uint32_t t = 0; t < kStatWords; t++) st[t] = part[t];
    for (uint32_t b = 1; b < sb; b++) {
        const uint64_t *q = &part[(size_t)b * kStatWords];
        st[0] = q[0] > st[0] ? q[0] : st[0];
        st[1] = q[1] < st[1] ? q[1] : st[1];
        for (uint32_t t = 2; t < kStatWords; t += 2) {
            st[t] |= q[t];
            st[t + 1] &= q[t + 1];
        }
    }
    const uint32_t D = (uint32_t)((st[0] + 7) / 8), minlen = (uint32_t)st[1];
    if (D > kMaxChunks) return LSM_EINVAL;
    std::vector<uint64_t> orand(2 * (size_t)(D > kFastChunks ? D : kFastChunks));
    for (uint32_t d = 0; d < kFastChunks; d++) {
        orand[2 * d] = st[4 + 2 * d];
        orand[2 * d + 1] = st[5 + 2 * d];
    }
    if (D > kFastChunks) {  // long keys: the remaining chunks by atomics
        uint64_t *dev = w.stats + 2;
        for (uint32_t d = kFastChunks; d < D; d++) {
            orand[2 * d] = 0;
            orand[2 * d + 1] = ~0ull;
        }
        LSM_HIP_CHECK(hipMemcpyAsync(dev, orand.data(), orand.size() * 8, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(merge_long_stats_kernel, dim3(sb), dim3(kMergeThreads), 0, s, m, D, dev);
        LSM_HIP_CHECK(hipMemcpyAsync(orand.data() + 2 * kFastChunks, dev + 2 * kFastChunks,
                                     (orand.size() - 2 * kFastChunks) * 8, hipMemcpyDeviceToHost, s));
        LSM_HIP_CHECK(hipStreamSynchronize(s));
    }

    // 2. stable LSD passes over packed groups of fields: from the least
    //    significant field (the key length) up to chunk 0; a group holds up
    //    to 64 varying bits
    std::vector<std::pair<uint32_t, uint64_t>> fields;  // least significant first
    if (st[2] & ~st[3]) fields.push_back({kNone, st[2] & ~st[3]});
    for (uint32_t d = D; d-- > 0;) {
        const uint64_t and_d = minlen > 8 * d ? orand[2 * d + 1] : 0;  // short keys hold 0
        const uint64_t vary = orand[2 * d] & ~and_d;
        if (vary) fields.push_back({d, vary});
    }
    int cur = 0;
    bool have_perm = false;
    for (size_t f0 = 0; f0 < fields.size();) {
        size_t f1 = f0;
        uint32_t bits = 0;
        while (f1 < fields.size() && f1 - f0 < kGroupFields &&
               bits + __builtin_popcountll(fields[f1].second) <= 64)
            bits += __builtin_popcountll(fields[f1++].second);
        SortGroup g{};
        g.nf = (uint32_t)(f1 - f0);
        for (size_t t = 0; t < g.nf; t++) {  // most significant first
            g.field[t] = fields[f1 - 1 - t].first;
            g.mask[t] = fields[f1 - 1 - t].second;
        }
        const bool k32 = bits <= 32;
        uint32_t *keys32[2] = {reinterpret_cast<uint32_t *>(w.keys[0]),
                               reinterpret_cast<uint32_t *>(w.keys[1])};
        if (k32)
            hipLaunchKernelGGL(merge_extract_kernel<uint32_t>, dim3(grid_for(n)), dim3(kMergeThreads),
                               0, s, m, have_perm ? w.perm[cur] : nullptr, g, keys32[0]);
        else
            hipLaunchKernelGGL(merge_extract_kernel<uint64_t>, dim3(grid_for(n)), dim3(kMergeThreads),
                               0, s, m, have_perm ? w.perm[cur] : nullptr, g, w.keys[0]);
        if (!have_perm) {
            hipLaunchKernelGGL(merge_iota_kernel, dim3(grid_for(n)), dim3(kMergeThreads), 0, s,
                               w.perm[cur], N);
            have_perm = true;
        }
        size_t tb = w.sort_bytes;
        const hipError_t e =
            k32 ? rocprim::radix_sort_pairs(w.sort_tmp, tb, keys32[0], keys32[1], w.perm[cur],
                                            w.perm[cur ^ 1], N, 0, bits, s)
                : rocprim::radix_sort_pairs(w.sort_tmp, tb, w.keys[0], w.keys[1], w.perm[cur],
                                            w.perm[cur ^ 1], N, 0, bits, s);
        if (e != hipSuccess) return -(1000 + (int)e);
        cur ^= 1;
        f0 = f1;
    }
    if (!have_perm)
        hipLaunchKernelGGL(merge_iota_kernel, dim3(grid_for(n)), dim3(kMergeThreads), 0, s,
                           w.perm[cur], N);
    const uint32_t *perm = w.perm[cur];

    if (tie == LSM_TIE_GOHEAP) {
        // container/heap's own tie order: dense key ranks from the sorted
        // order (equal-to-predecessor flags on the device), the heap's
        // push / pop history replayed over the ranks on this thread, and
        // its pop order -- sorted by key, equal keys as the heap pops them
        // -- becomes the sorted order the steps below walk
        hipLaunchKernelGGL(merge_eq_kernel, dim3(grid_for(n)), dim3(kMergeThreads), 0, s, m, perm,
                           w.flags);
        LSM_HIP_CHECK(hipGetLastError());
        std::vector<uint32_t> hperm(N), rank(N), order(N);
        std::vector<uint8_t> eq(N);
        LSM_HIP_CHECK(hipMemcpyAsync(hperm.data(), perm, 4ull * N, hipMemcpyDeviceToHost, s));
        LSM_HIP_CHECK(hipMemcpyAsync(eq.data(), w.flags, N, hipMemcpyDeviceToHost, s));
        LSM_HIP_CHECK(hipStreamSynchronize(s));
        uint32_t g = 0;
        for (uint32_t j = 0; j < N; j++) {
            g += (j > 0 && !eq[j]) ? 1u : 0u;
            rank[hperm[j]] = g;
        }
        goheap_pop_order(rank.data(), N, order.data());
        LSM_HIP_CHECK(hipMemcpyAsync(w.perm[cur], order.data(), 4ull * N, hipMemcpyHostToDevice, s));
        LSM_HIP_CHECK(hipStreamSynchronize(s));  // `order` is freed on return
    }

    // 3. groups and candidates; 4. sums and the file walk; 5. emit
    hipLaunchKernelGGL(merge_flags_kernel, dim3(grid_for(n)), dim3(kMergeThreads), 0, s, m, perm,
                       level, w.flags, w.csize);
    hipLaunchKernelGGL(merge_candidate_kernel, dim3(grid_for(n)), dim3(kMergeThreads), 0, s, m,
                       w.flags, w.csize);
    const uint32_t ntiles = (N + kScanTile - 1) / kScanTile;
    hipLaunchKernelGGL(merge_scan_tiles, dim3(ntiles), dim3(kMergeThreads), 0, s, w.csize, N,
                       w.scan_part);
    hipLaunchKernelGGL(merge_scan_partials, dim3(1), dim3(kMergeThreads), 0, s, w.scan_part, ntiles,
                       w.sc, N);
    hipLaunchKernelGGL(merge_scan_apply, dim3(ntiles), dim3(kMergeThreads), 0, s, w.csize, N,
                       w.scan_part, w.sc);
    WalkArgs wa{m, perm, w.flags, w.sc, threshold, w.files, d_out, w.stats};
    hipLaunchKernelGGL(merge_walk_kernel, dim3(1), dim3(64), 0, s, wa);
    hipLaunchKernelGGL(merge_emit_kernel, dim3(grid_for(n + 1)), dim3(kMergeThreads), 0, s, perm,
                       w.sc, w.csize, w.files, w.stats, N, d_out, d_file_start);
    LSM_HIP_CHECK(hipGetLastError());
    uint64_t c3[3];
    LSM_HIP_CHECK(hipMemcpyAsync(c3, w.stats, sizeof c3, hipMemcpyDeviceToHost, s));
    LSM_HIP_CHECK(hipStreamSynchronize(s));
    for (int i = 0; i < 3; i++) h_counts[i] = c3[i];
    return 0;
}

extern "C" int lsm_merge_kvs(lsm_ctx *ctx, const uint8_t *d_bytes, const lsm_rec_desc *d_key_desc,
                             const lsm_rec_desc *d_val_desc, uint64_t n, int level,
                             uint64_t threshold, uint32_t *d_out, uint64_t *d_file_start,
                             uint64_t *h_counts, void *d_ws, size_t ws_bytes, void *stream) {
    // the v2 / v3 contract: exactly two counts, {nout, nfiles}; only
    // lsm_merge_kvs_tie reports the third (the most pairs in one file)
    if (!h_counts) return LSM_EINVAL;
    uint64_t c3[3] = {0, 0, 0};
    const int rc = lsm_merge_kvs_tie(ctx, d_bytes, d_key_desc, d_val_desc, n, level, threshold,
                                     LSM_TIE_INPUT, d_out, d_file_start, c3, d_ws, ws_bytes, stream);
    h_counts[0] = c3[0];
    h_counts[1] = c3[1];
    return rc;
}

extern "C" size_t lsm_gather_kvs_workspace_bytes(uint64_t nout) {
    const size_t nn = nout ? nout : 1;
    const size_t ntiles = (nn + kScanTile - 1) / kScanTile;
    return 2 * ((4 * nn + 255) & ~(size_t)255) + 8 * ntiles + 256;
}

namespace lsm {
int scan_u32_to_u64(const uint32_t *d_len, uint32_t n, uint64_t *d_out, void *ws, size_t ws_bytes,
                    hipStream_t s);
}

extern "C" int lsm_gather_kvs(lsm_ctx *ctx, const uint8_t *d_bytes, const lsm_rec_desc *d_key_desc,
                              const lsm_rec_desc *d_val_desc, const uint32_t *d_idx, uint64_t nout,
                              uint8_t *d_keys, uint64_t *d_koff, uint8_t *d_vals, uint64_t *d_voff,
                              void *d_ws, size_t ws_bytes, void *stream) {
    if (!ctx || !d_koff || !d_voff || nout >= 0xFFFFFFFFull) return LSM_EINVAL;
    if (nout && (!d_bytes || !d_key_desc || !d_idx || !d_keys || !d_ws)) return LSM_EINVAL;
    if (ws_bytes < lsm_gather_kvs_workspace_bytes(nout)) return LSM_ESPACE;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint32_t N = (uint32_t)nout;
    const size_t nn = nout ? nout : 1, part = (4 * nn + 255) & ~(size_t)255;
    uint32_t *kl = static_cast<uint32_t *>(d_ws);
    uint32_t *vl = reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(d_ws) + part);
    void *sw = static_cast<uint8_t *>(d_ws) + 2 * part;
    const size_t sbytes = ws_bytes - 2 * part;
    const MergeIn m{d_bytes, d_key_desc, d_val_desc, N};
    if (N)
        hipLaunchKernelGGL(gather_lens_kernel, dim3(grid_for(nout)), dim3(kMergeThreads), 0, s, m,
                           d_idx, N, kl, vl);
    int rc = scan_u32_to_u64(kl, N, d_koff, sw, sbytes, s);
    if (!rc) rc = scan_u32_to_u64(vl, N, d_voff, sw, sbytes, s);
    if (rc) return rc;
    if (N)
        hipLaunchKernelGGL(gather_copy_kernel, dim3((N + kMergeThreads - 1) / kMergeThreads),
                           dim3(kMergeThreads), 0, s, m, d_idx, N, d_koff, d_voff, d_keys, d_vals);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}

extern "C" int lsm_sst_image_sizes(lsm_ctx *ctx, const uint64_t *d_koff, const uint64_t *d_voff,
                                   const uint64_t *d_file_start, uint32_t nfile, uint64_t m,
                                   uint64_t *d_size, void *stream) {
    if (!ctx || (nfile && (!d_koff || !d_voff || !d_file_start || !d_size))) return LSM_EINVAL;
    if (nfile == 0) return 0;
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(sst_sizes_kernel, dim3(grid_for(nfile)), dim3(kMergeThreads), 0, s, d_koff,
                       d_voff, d_file_start, nfile, lsm_filter_block_size(m), d_size);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}

extern "C" int lsm_sst_layout(lsm_ctx *ctx, const uint64_t *d_koff, const uint64_t *d_voff,
                              const uint64_t *d_file_start, uint32_t nfile, uint64_t m,
                              uint32_t align, uint64_t *d_size, uint64_t *d_file_off,
                              void *stream) {
    if (!ctx || align == 0 || !d_file_off) return LSM_EINVAL;
    if (nfile && (!d_koff || !d_voff || !d_file_start || !d_size)) return LSM_EINVAL;
    hipLaunchKernelGGL(sst_layout_kernel, dim3(1), dim3(kMergeThreads), 0,
                       static_cast<hipStream_t>(stream), d_koff, d_voff, d_file_start, nfile,
                       lsm_filter_block_size(m), (uint64_t)align, d_size, d_file_off);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}

extern "C" int lsm_sst_pairs(lsm_ctx *ctx, const lsm_sst_meta *d_meta, const uint64_t *d_file_off,
                             uint32_t nfile, const lsm_rec_desc *d_idx_desc,
                             const lsm_rec_desc *d_data_desc, lsm_rec_desc *d_key_out,
                             lsm_rec_desc *d_val_out, uint64_t *d_prefix, void *stream) {
    if (!ctx || !d_prefix) return LSM_EINVAL;
    if (nfile && (!d_meta || !d_file_off || !d_idx_desc || !d_data_desc || !d_key_out || !d_val_out))
        return LSM_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(sst_pairs_scan_kernel, dim3(1), dim3(kMergeThreads), 0, s, d_meta, nfile,
                       d_prefix);
    if (nfile)
        hipLaunchKernelGGL(sst_pairs_copy_kernel, dim3(16, nfile), dim3(kMergeThreads), 0, s, d_meta,
                           d_file_off, reinterpret_cast<const u32x4 *>(d_idx_desc),
                           reinterpret_cast<const u32x4 *>(d_data_desc), d_prefix,
                           reinterpret_cast<u32x4 *>(d_key_out), reinterpret_cast<u32x4 *>(d_val_out));
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}
