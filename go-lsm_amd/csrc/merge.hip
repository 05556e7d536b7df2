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
//      one workgroup walks the file boundaries -- the windows around the next
//      kWalkWins files' predicted ends are loaded in one round trip and the
//      chain runs through them in LDS; a flush inside a group makes the next
//      writable pair of that group a write of its own (the "extra" of the
//      next file);
//   5. emit: each candidate's output slot from its file's start.
// Steps 3-5 are exact for any input; only the tie order is specified above.

#include <rocprim/device/device_radix_sort.hpp>

#include <cstdio>
#include <cstdlib>
#include <chrono>
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
constexpr uint32_t kMergePathMin = 4096;  // fewer pairs: the radix passes alone

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

// plain loads: the stats, flags, rank and gather passes read the same
// descriptors again (nt loads: compaction 1.027 -> 1.018 ms without them, A/B)
__device__ __forceinline__ View view(const MergeIn &m, uint32_t i) {
    const u32x4 k = reinterpret_cast<const u32x4 *>(m.kd)[i];
    View v;
    v.ko = ((uint64_t)k.y << 32 | k.x) + 4;
    v.kl = k.z;
    if (m.vd) {
        const u32x4 d = reinterpret_cast<const u32x4 *>(m.vd)[i];
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
__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t l) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)l) << 32 |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)l);
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

// Go string order of two keys (bytes.Compare / string <): big-endian 8-byte
// chunks zero padded past the shorter key, then the lengths.
__device__ __forceinline__ int key_cmp(const uint8_t *b, const View &x, const View &y) {
    const uint32_t l = x.kl > y.kl ? x.kl : y.kl;
    for (uint32_t d = 0; 8 * d < l; d++) {
        const uint64_t cx = key_chunk(b + x.ko, x.kl, d), cy = key_chunk(b + y.ko, y.kl, d);
        if (cx != cy) return cx < cy ? -1 : 1;
    }
    return x.kl < y.kl ? -1 : x.kl > y.kl ? 1 : 0;
}

// Per-block partial statistics over a contiguous tile of the input: [0] max
// key length, [1] min key length, [2] OR / [3] AND of the key lengths, then
// for chunks d < kFastChunks the OR and AND of chunk d over keys longer than
// 8d (shorter keys hold 0 there: the host folds that in with the minimum key
// length); then the tile's run summary (sorted runs of the input, a run
// breaking at each descent key(i) < key(i - 1)): the first and last descent,
// their count and, when the tile holds at most 64 descents, its longest run
// strictly inside the tile -- the host picks the input's longest sorted run
// from these (the merge path, merge_kvs_impl).
constexpr uint32_t kStatCore = 4 + 2 * kFastChunks;
constexpr uint32_t kStatWords = kStatCore + 5;

__global__ __launch_bounds__(kMergeThreads) void merge_stats_kernel(MergeIn m, uint32_t chunk,
                                                                    uint64_t *part) {
    __shared__ uint64_t red[kMergeThreads / kWave][kStatCore];
    __shared__ uint32_t s_desc[kWave];
    __shared__ uint32_t s_first, s_last, s_cnt;
    uint64_t s[kStatCore];
    s[0] = 0; s[1] = ~0ull; s[2] = 0; s[3] = ~0ull;
    for (uint32_t d = 0; d < kFastChunks; d++) {
        s[4 + 2 * d] = 0;
        s[5 + 2 * d] = ~0ull;
    }
    if (threadIdx.x == 0) {
        s_first = kNone;
        s_last = 0;
        s_cnt = 0;
    }
    __syncthreads();
    const uint32_t lo = blockIdx.x * chunk, hi = lo + chunk < m.n ? lo + chunk : m.n;
    for (uint32_t i = lo + threadIdx.x; i < hi; i += kMergeThreads) {
        const View v = view(m, i);
        s[0] = v.kl > s[0] ? v.kl : s[0];
        s[1] = v.kl < s[1] ? v.kl : s[1];
        s[2] |= v.kl;
        s[3] &= v.kl;
        uint64_t ch[kFastChunks];
#pragma unroll
        for (uint32_t d = 0; d < kFastChunks; d++) {
            ch[d] = v.kl > 8 * d ? key_chunk(m.bytes + v.ko, v.kl, d) : 0;
            if (v.kl > 8 * d) {
                s[4 + 2 * d] |= ch[d];
                s[5 + 2 * d] &= ch[d];
            }
        }
        // the predecessor's first 32 bytes from the lane below (its key was
        // loaded there; lane 0 loads it): the descent test compares chunks,
        // and the whole keys only when those tie and a key is longer
        uint64_t pc[kFastChunks];
        uint32_t pkl = __shfl_up(v.kl, 1);
#pragma unroll
        for (uint32_t d = 0; d < kFastChunks; d++) pc[d] = __shfl_up(ch[d], 1);
        if (lane_id() == 0 && i > 0) {
            const View u = view(m, i - 1);
            pkl = u.kl;
#pragma unroll
            for (uint32_t d = 0; d < kFastChunks; d++)
                pc[d] = u.kl > 8 * d ? key_chunk(m.bytes + u.ko, u.kl, d) : 0;
        }
        int cmp = 0;
#pragma unroll
        for (uint32_t d = 0; d < kFastChunks; d++)
            if (cmp == 0 && ch[d] != pc[d]) cmp = ch[d] < pc[d] ? -1 : 1;
        if (cmp == 0 && i > 0) {
            if (v.kl <= 8 * kFastChunks && pkl <= 8 * kFastChunks) cmp = v.kl < pkl ? -1 : v.kl > pkl ? 1 : 0;
            else cmp = key_cmp(m.bytes, v, view(m, i - 1));
        }
        if (i > 0 && cmp < 0) {  // a descent: a run starts at i
            atomicMin(&s_first, i);
            atomicMax(&s_last, i);
            const uint32_t at = atomicAdd(&s_cnt, 1u);
            if (at < kWave) s_desc[at] = i;
        }
    }
    s[0] = wave_max64(s[0]);
    s[1] = wave_min64(s[1]);
    for (uint32_t t = 2; t < kStatCore; t += 2) {
        s[t] = wave_or64(s[t]);
        s[t + 1] = wave_and64(s[t + 1]);
    }
    const uint32_t w = threadIdx.x / kWave;
    if (lane_id() == 0)
        for (uint32_t t = 0; t < kStatCore; t++) red[w][t] = s[t];
    __syncthreads();
    uint64_t *out = part + (uint64_t)blockIdx.x * kStatWords;
    if (threadIdx.x < kStatCore) {
        const uint32_t t = threadIdx.x;
        uint64_t r = red[0][t];
        for (uint32_t x = 1; x < kMergeThreads / kWave; x++) {
            const uint64_t y = red[x][t];
            if (t == 0) r = y > r ? y : r;
            else if (t == 1) r = y < r ? y : r;
            else if (t & 1) r &= y;
            else r |= y;
        }
        out[t] = r;
    }
    if (w == 1) {
        // the longest run between two of the tile's descents (<= 64 of them)
        const uint32_t cnt = s_cnt, lane = lane_id();
        uint64_t bs = 0, be = 0;
        if (cnt >= 2 && cnt <= kWave) {
            const uint32_t x = lane < cnt ? s_desc[lane] : kNone;
            uint32_t nx = kNone;  // the next descent after x
            for (uint32_t l = 0; l < cnt; l++) {
                const uint32_t y = (uint32_t)__builtin_amdgcn_readlane((int)x, (int)l);
                if (y > x && y < nx) nx = y;
            }
            const uint64_t len = lane < cnt && nx != kNone ? (uint64_t)(nx - x) : 0;
            const uint64_t key = len << 32 | x;
            const uint64_t best = wave_max64(key);
            bs = (uint32_t)best;
            be = bs + (best >> 32);
        }
        if (lane == 0) {
            out[kStatCore + 0] = s_first;
            out[kStatCore + 1] = s_last;
            out[kStatCore + 2] = cnt;
            out[kStatCore + 3] = bs;
            out[kStatCore + 4] = be;
        }
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

// The merge path (one sorted run holds most pairs -- a level-1 run with a
// few level-0 files merged into it): the pairs outside the run are sorted by
// the radix passes, and every pair's sorted position is its rank in its own
// sequence plus its rank in the other, by (packed key, input index) --
// stable, exactly the order the LSD passes give, in one pass over the run.
// packed key of pair i (as merge_extract_kernel)
template <class K>
__device__ __forceinline__ K packed_key(const MergeIn &m, const SortGroup &g, uint32_t i) {
    const View v = view(m, i);
    uint64_t key = 0;
    for (uint32_t t = 0; t < g.nf; t++) {
        const uint64_t x = g.field[t] == kNone ? v.kl : key_chunk(m.bytes + v.ko, v.kl, g.field[t]);
        const uint32_t bits = (uint32_t)__builtin_popcountll(g.mask[t]);
        key = (bits >= 64 ? 0 : key << bits) | pext64(x, g.mask[t]);
    }
    return (K)key;
}

// the run [s, e): keys[r] = key of s + r; the others: keys[j], idx[j] of the
// j-th pair outside the run (input order)
template <class K>
__global__ __launch_bounds__(kMergeThreads) void merge_extract_split_kernel(MergeIn m, SortGroup g,
                                                                            uint32_t s, uint32_t e,
                                                                            K *run_keys, K *oth_keys,
                                                                            uint32_t *oth_idx, uint32_t *zero) {
    const uint32_t j = blockIdx.x * kMergeThreads + threadIdx.x;
    if (j == 0 && zero) *zero = 0;  // the k-way path's run-start count
    if (j >= m.n) return;
    if (j >= s && j < e) {
        run_keys[j - s] = packed_key<K>(m, g, j);
    } else {
        const uint32_t q = j < s ? j : j - (e - s);
        oth_keys[q] = packed_key<K>(m, g, j);
        oth_idx[q] = j;
    }
}

// sorted position of run pair s + r: r + the others before it
template <class K>
__global__ __launch_bounds__(kMergeThreads) void merge_rank_run_kernel(const K *run_keys, uint32_t nrun,
                                                                       uint32_t s, const K *ok,
                                                                       const uint32_t *oi, uint32_t no,
                                                                       uint32_t *perm) {
    const uint32_t r = blockIdx.x * kMergeThreads + threadIdx.x;
    if (r >= nrun) return;
    const K k = run_keys[r];
    const uint32_t i = s + r;
    uint32_t lo = 0, hi = no;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const K x = ok[mid];
        if (x < k || (x == k && oi[mid] < i)) lo = mid + 1;
        else hi = mid;
    }
    perm[r + lo] = i;
}

// sorted position of the q-th sorted other: q + the run pairs before it
template <class K>
__global__ __launch_bounds__(kMergeThreads) void merge_rank_others_kernel(const K *run_keys, uint32_t nrun,
                                                                          uint32_t s, const K *ok,
                                                                          const uint32_t *oi, uint32_t no,
                                                                          uint32_t *perm) {
    const uint32_t q = blockIdx.x * kMergeThreads + threadIdx.x;
    if (q >= no) return;
    const K k = ok[q];
    const uint32_t i = oi[q];
    uint32_t lo = 0, hi = nrun;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const K x = run_keys[mid];
        if (x < k || (x == k && s + mid < i)) lo = mid + 1;
        else hi = mid;
    }
    perm[q + lo] = i;
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
//
// xinfo[j] = perm[j] | writable << 32 | min(EstimateSize, 2^24 - 1) << 40:
// what merge_scan_apply needs of a file's extra (usually the pair right after
// a candidate) in one load.
__global__ __launch_bounds__(kMergeThreads) void merge_flags_kernel(MergeIn m, const uint32_t *perm,
                                                                    int level, uint8_t *flags,
                                                                    uint32_t *csize, uint64_t *xinfo) {
    const uint32_t j = blockIdx.x * kMergeThreads + threadIdx.x;
    if (j >= m.n) return;
    const uint32_t pj = perm[j];
    const View v = view(m, pj);
    bool gs = j == 0 || v.kl == 0;
    if (!gs) gs = !keys_equal(m.bytes, v, view(m, perm[j - 1]));
    const bool wr = level < 6 || !is_tombstone(m.bytes, v);
    flags[j] = (uint8_t)((gs ? 1 : 0) | (wr ? 2 : 0));
    const uint64_t sz = 16 + (uint64_t)v.kl + v.vl;
    csize[j] = (uint32_t)sz;
    xinfo[j] = (uint64_t)pj | (uint64_t)(wr ? 1 : 0) << 32 | (sz < 0xFFFFFFull ? sz : 0xFFFFFFull) << 40;
}

// eq[j] = 1 when sorted position j holds the same key as j - 1 (plain key
// equality: for container/heap "" equals "", merge.go:21-23's Less is key <)
// LSM_TIE_GOHEAP's dense key ranks, on the device: newg[j] = 1 where sorted
// position j starts a new key (merge_scan_tiles / merge_scan_partials then
// give each tile its first rank), and goheap_rank_apply writes each pair's
// rank by input index -- the only array the host's heap replay reads.
__global__ __launch_bounds__(kMergeThreads) void goheap_newgroup_kernel(MergeIn m, const uint32_t *perm,
                                                                        uint32_t *newg) {
    const uint32_t j = blockIdx.x * kMergeThreads + threadIdx.x;
    if (j >= m.n) return;
    newg[j] = j > 0 && !keys_equal(m.bytes, view(m, perm[j]), view(m, perm[j - 1]));
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

// one pass over the tile sums by 1,024 threads (see plan_scan_partials): a
// contiguous stretch per thread, one block scan of the stretch sums
constexpr uint32_t kPartThreads = 1024;

__global__ __launch_bounds__(kPartThreads) void merge_scan_partials(SumPair *part, uint32_t ntiles,
                                                                    SumPair *sc, uint32_t n) {
    __shared__ uint64_t ws_[kPartThreads / kWave], wc_[kPartThreads / kWave];
    const uint32_t per = (ntiles + kPartThreads - 1) / kPartThreads, b = threadIdx.x * per;
    const uint32_t e = b + per < ntiles ? b + per : ntiles;
    uint64_t s = 0, c = 0;
    for (uint32_t i0 = b; i0 < e; i0 += 8) {  // 8 loads in flight
        SumPair v[8];
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) v[k] = i0 + k < e ? part[i0 + k] : SumPair{0, 0};
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) {
            s += v[k].s;
            c += v[k].c;
        }
    }
    uint64_t ts, tc;
    const uint64_t xs = wave_excl_scan64(s, &ts), xc = wave_excl_scan64(c, &tc);
    const uint32_t w = threadIdx.x / kWave;
    if (lane_id() == 0) {
        ws_[w] = ts;
        wc_[w] = tc;
    }
    __syncthreads();
    SumPair pre{xs, xc}, tot{0, 0};
    for (uint32_t i = 0; i < kPartThreads / kWave; i++) {
        if (i < w) {
            pre.s += ws_[i];
            pre.c += wc_[i];
        }
        tot.s += ws_[i];
        tot.c += wc_[i];
    }
    for (uint32_t i0 = b; i0 < e; i0 += 8) {
        SumPair v[8];
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) v[k] = i0 + k < e ? part[i0 + k] : SumPair{0, 0};
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) {
            if (i0 + k < e) part[i0 + k] = pre;
            pre.s += v[k].s;
            pre.c += v[k].c;
        }
    }
    if (threadIdx.x == 0) sc[n] = tot;
}

__global__ __launch_bounds__(kMergeThreads) void goheap_rank_apply(const uint32_t *newg, uint32_t n,
                                                                   const SumPair *part,
                                                                   const uint32_t *perm,
                                                                   uint32_t *rank) {
    uint32_t f[kScanPer];
    uint64_t s = 0;
    const uint64_t i0 = (uint64_t)blockIdx.x * kScanTile + threadIdx.x * kScanPer;
    for (uint32_t t = 0; t < kScanPer; t++) {
        f[t] = i0 + t < n ? newg[i0 + t] : 0u;
        s += f[t];
    }
    SumPair tot;
    const SumPair x = block_excl_scan2(s, 0, &tot);
    uint64_t g = x.s + part[blockIdx.x].s;
    for (uint32_t t = 0; t < kScanPer; t++) {
        g += f[t];  // inclusive: the rank of position i0 + t
        if (i0 + t < n) rank[perm[i0 + t]] = (uint32_t)g;
    }
}

// The sums per position, and per candidate c (the walk's plateau space, see
// merge_walk_kernel): cand_pn[c] = the size sum after it, cand_pos[c] = its
// position | 1 << 31 when the position after it continues its group, and for
// such a candidate cand_ext[c]: the extra of the file that would start there
// (the group's next writable pair, merge.go:67-72 after lastWrittenKey's
// reset) as perm value | (its position - c's) << 32 | its EstimateSize << 40;
// position delta 0: the group ends with no writable pair; 255: not resolved
// within kExtScan positions, or a pair of 2^24 bytes or more (the walk's
// general step).
constexpr uint32_t kExtScan = 254;

__global__ __launch_bounds__(kMergeThreads) void merge_scan_apply(const uint32_t *csize, uint32_t n,
                                                                  const SumPair *part, SumPair *sc,
                                                                  const uint8_t *flags, MergeIn m,
                                                                  const uint32_t *perm, const uint64_t *xinfo,
                                                                  uint64_t *cand_pn,
                                                                  uint32_t *cand_pos, uint64_t *cand_ext) {
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
        if (v[t]) {
            const uint64_t k = i0 + t;
            const bool cont = k + 1 < n && !(flags[k + 1] & 1);
            cand_pn[pc] = ps + v[t];
            cand_pos[pc] = (uint32_t)k | (cont ? 0x80000000u : 0u);
            if (cont) {
                uint64_t X = 0xFFull << 32;
                const uint64_t x1 = xinfo[k + 1];  // usually the extra itself
                if ((x1 >> 32) & 1) {
                    const uint64_t sz = x1 >> 40;
                    if (sz < 0xFFFFFFull) X = (x1 & 0xFFFFFFFFull) | 1ull << 32 | sz << 40;
                } else for (uint32_t d = 2; d <= kExtScan; d++) {
                    const uint64_t q = k + d;
                    const uint8_t f = q < n ? flags[q] : 1;
                    if (f & 1) {  // the group ends with no writable pair
                        X = 0;
                        break;
                    }
                    if (f & 2) {
                        const uint32_t wq = perm[q];
                        const View w = view(m, wq);
                        const uint64_t sz = 16 + (uint64_t)w.kl + w.vl;
                        if (sz < (1ull << 24)) X = (uint64_t)wq | (uint64_t)d << 32 | sz << 40;
                        break;
                    }
                }
                cand_ext[pc] = X;
            }
        }
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
    const uint64_t *cand_pn;   // per candidate: the size sum after it
    const uint32_t *cand_pos;  // per candidate: its position | continues << 31
    const uint64_t *cand_ext;  // per continuing candidate: the next file's extra (merge_scan_apply)
    const uint8_t *abs_succ;   // merge_walk_abs_kernel's maps, window bases and head
    const uint64_t *abs_bases;
    const uint32_t *abs_head;
    uint64_t threshold;
    MergeFile *files;
    uint32_t *out;
    uint64_t *counts;   // [0] = written pairs, [1] = files, [2] = most pairs in one file
};

// The file walk (merge.go:57-91): file f starts at sorted position p; if p
// continues a group whose pair was written just before the flush,
// lastWrittenKey is "" again and the group's next writable pair is written
// (the file's "extra"); then come the candidates of later groups until the
// size reaches the threshold.  The chain of files is sequential, so its cost
// is the round trips it waits on.  One workgroup walks it.
//
// Plateau space.  S(k), the candidate sizes before position k, is flat across
// non-candidates, and a file ends at the first k > g with S(k) >= its target:
// the position after a candidate.  With P[e] the size sum of the first e
// candidates (cand_pn[e - 1]), a file whose first candidate is e0 writes its
// extra (if any) and candidates e0 .. e - 1, e = the first plateau with
// P[e] >= P[e0] + T - (the extra's size), and the next file starts at
// cand_pos[e - 1] + 1 -- a group start unless that candidate's group goes on
// (cand_pos bit 31; its extra is then in cand_ext[e - 1]).  Duplicates and
// dropped tombstones take no plateau, so a file's plateau count is its pair
// count and varies only with the pair sizes.
//  * prediction: each round loads, in one round trip by the whole
//    workgroup, a window of W = kWalkEntries / R plateaus around the
//    predicted end of each of the next R files (file r of the round ends near
//    e0 + (r + 1) * span, span = the mean pairs per file so far) into LDS;
//  * succession (all threads, LDS only): every plateau of window r, taken as
//    the start of file r + 1, gets that file's end in window r + 1 by a
//    binary search -- exact when the plateau before it is in the window
//    (below the target there) or is the file's own start;
//  * chain (wave 0): file 0's end by ballots over window 0, then one LDS
//    lookup per file;
//  * a file whose end falls outside its window ends the round, and the next
//    round predicts fewer files in wider windows (a round that resolves all
//    its files doubles R); a continuation whose extra was not resolved by
//    merge_scan_apply, a pair as large as the threshold, or an end outside a
//    one-file window is walked by the whole workgroup (group end and extra
//    by a parallel scan of the flags, the end by a 1,024-way search over S).
// Round 3's one-wave walk (position windows, 8 files per round trip) took
// 160 us for 208 files; a position-window form with 12 files per round,
// 470 us (the duplicates' position drift missed its windows).
constexpr uint32_t kWalkThreads = 1024;
constexpr uint32_t kWalkEntries = 4 * kWalkThreads;  // window plateaus per round
constexpr uint32_t kWalkMaxR = 32;                   // most files predicted per round
constexpr uint16_t kSuccMiss = 0xFFFF, kSuccGeneral = 0xFFFE, kSuccStop = 0xFFFD,
                   kSuccLast = 0xFFFC;

struct WalkState {
    uint32_t p, e, nf, span, R, stop;  // e = C(p); stop: 1 = walk done, 2 = general step next
    uint64_t o, most, P;               // P = S(p)
};

// The file that starts right after plateau e (P = P[e], Q = cand_pos[e - 1],
// X = cand_ext[e - 1]; first = the walk's first file, at 0): its first
// position p, its extra (wpos / wperm, kNone if none) and its target, or the
// code of a file the window search does not resolve.
__device__ __forceinline__ uint16_t walk_file(uint64_t P, uint32_t Q, uint64_t X, bool first, uint32_t n,
                                              uint64_t T, uint64_t tail_s, uint32_t &p, uint32_t &wpos,
                                              uint32_t &wperm, uint64_t &tg) {
    wpos = kNone;
    wperm = 0;
    uint64_t wsize = 0;
    p = 0;
    if (!first) {
        p = (Q & 0x7FFFFFFFu) + 1;
        if (p >= n) return kSuccStop;
        if (Q >> 31) {  // continues a group
            const uint32_t d = (uint32_t)(X >> 32) & 0xFFu;
            if (d == 0xFFu) return kSuccGeneral;
            if (d) {
                wpos = (Q & 0x7FFFFFFFu) + d;
                wperm = (uint32_t)X;
                wsize = X >> 40;
                if (wsize >= T) return kSuccGeneral;  // the extra alone fills the file
            }
        }
    }
    tg = P + T - wsize;
    return tail_s < tg ? kSuccLast : 0;
}

// ---- one-shot prediction of every file's end ------------------------------
//
// Before the rounds, merge_walk_abs_kernel predicts the end of every file of
// the walk at once, from plateau 0: file f of a uniform stream ends near
// plateau (f + 1) * span, span = (T + half a mean pair) / the mean pair (the
// overshoot past T is half a pair on average), and the deviation only
// accumulates the files' varying pair counts (a random walk: on the
// compaction bench within +-55 plateaus over 208 files).  One workgroup per
// window of kAbsW plateaus around each predicted end maps every plateau of
// its window, taken as the end of file f, to file f + 1's end in the next
// window (the same exact test as a round's succession), and the walk chains
// the maps from file 0 in LDS.  The first miss (or a window limit) hands the
// rest of the walk to the rounds.
constexpr uint32_t kAbsW = 248;      // plateaus per window
constexpr uint32_t kAbsThreads = 256;
constexpr uint8_t kAbsLast = 252, kAbsStop = 253, kAbsGeneral = 254, kAbsMiss = 255;
constexpr uint32_t kAbsMaxWin = 352;  // files predicted: 352 x 248 B of the walk's LDS

struct AbsArgs {
    const uint64_t *cand_pn;
    const uint32_t *cand_pos;
    const uint64_t *cand_ext;
    const SumPair *sc;
    uint32_t n;
    uint64_t threshold;
    uint8_t *succ;    // [kAbsMaxWin][kAbsW]
    uint64_t *bases;  // [kAbsMaxWin][2]: window f's first plateau, and window f + 1's as block f used it
    uint32_t *head;   // [0] = windows, [1] = file 0's end in window 0 (or a code)
};

__device__ __forceinline__ uint32_t abs_windows(const SumPair &tail, uint64_t T) {
    if (tail.c == 0) return 0;
    const uint64_t nf = tail.s / T + 2;
    return nf < kAbsMaxWin ? (uint32_t)nf : kAbsMaxWin;
}
__device__ __forceinline__ uint64_t abs_base(const SumPair &tail, uint64_t T, uint32_t f) {
    const double span = ((double)T + 0.5 * (double)tail.s / (double)tail.c) * (double)tail.c / (double)tail.s;
    const uint64_t c = (uint64_t)((double)(f + 1) * span + 0.5);
    return c > 1 + kAbsW / 2 ? c - kAbsW / 2 : 1;
}

__global__ __launch_bounds__(kAbsThreads) void merge_walk_abs_kernel(AbsArgs a) {
    __shared__ uint64_t np[kAbsW];
    __shared__ uint32_t s_first;
    const uint32_t f = blockIdx.x, t = threadIdx.x;
    const SumPair tail = a.sc[a.n];
    const uint64_t T = a.threshold;
    const uint32_t nwin = abs_windows(tail, T), ncand = (uint32_t)tail.c;
    if (f == 0 && t == 0) a.head[0] = nwin;
    if (f >= nwin) return;
    const uint64_t b0 = abs_base(tail, T, f), b1 = abs_base(tail, T, f + 1);
    if (t == 0) s_first = kAbsW;
    uint64_t P = ~0ull, X = 0;
    uint32_t Q = 0;
    const uint64_t e = b0 + t;
    if (t < kAbsW) {
        const uint64_t e1 = b1 + t;
        np[t] = e1 <= ncand ? a.cand_pn[e1 - 1] : ~0ull;
        if (e <= ncand) {
            P = a.cand_pn[e - 1];
            Q = a.cand_pos[e - 1];
            X = a.cand_ext[e - 1];
        }
    }
    __syncthreads();
    if (f == 0 && t < kAbsW && P >= T) atomicMin(&s_first, t);  // file 0 ends at P >= T
    if (t < kAbsW) {
        uint8_t out = kAbsMiss;
        if (e <= ncand) {
            uint32_t p, wpos, wperm;
            uint64_t tg = ~0ull;
            const uint16_t c = walk_file(P, Q, X, false, a.n, T, tail.s, p, wpos, wperm, tg);
            if (c == kSuccLast) out = kAbsLast;
            else if (c == kSuccStop) out = kAbsStop;
            else if (c == kSuccGeneral) out = kAbsGeneral;
            else {
                uint32_t pos = 0;
                for (uint32_t s = 128; s > 0; s >>= 1)
                    if (pos + s <= kAbsW && np[pos + s - 1] < tg) pos += s;
                // pos = the first window-(f + 1) plateau at the target, or kAbsW
                if (pos < kAbsW && (pos > 0 || b1 <= e + 1)) out = (uint8_t)pos;
            }
        }
        a.succ[(uint64_t)f * kAbsW + t] = out;
    }
    if (t == 0) {
        a.bases[2 * f] = b0;
        a.bases[2 * f + 1] = b1;
    }
    __syncthreads();
    if (f == 0 && t == 0) {  // file 0 (from position 0, no extra): the target is T
        const uint32_t x = s_first;
        a.head[1] = tail.s < T ? kAbsLast : (x < kAbsW && (x > 0 || b0 <= 1)) ? x : kAbsMiss;
    }
}

__global__ __launch_bounds__(kWalkThreads) void merge_walk_kernel(WalkArgs a) {
    // the rounds' windows; phase 1's maps before them
    __shared__ __attribute__((aligned(16))) uint8_t lds_raw[kWalkEntries * 22];
    uint64_t *wp = reinterpret_cast<uint64_t *>(lds_raw);  // P of each window plateau
    uint64_t *wx = wp + kWalkEntries;                       // cand_ext of its last candidate
    uint32_t *wq = reinterpret_cast<uint32_t *>(wx + kWalkEntries);  // cand_pos of its last candidate
    uint16_t *sx = reinterpret_cast<uint16_t *>(wq + kWalkEntries);  // succession: the next file's end
    static_assert(kAbsMaxWin * kAbsW <= kWalkEntries * 22, "phase 1 maps fit the window buffers");
    __shared__ uint64_t s_bases[2 * kAbsMaxWin];
    __shared__ uint8_t s_chosen[kAbsMaxWin];
    __shared__ uint64_t s_wsum[kWalkThreads / kWave], s_wmax[kWalkThreads / kWave];
    __shared__ uint32_t s_nres, s_code;
    __shared__ WalkState st;
    __shared__ uint32_t s_min[2];
    __shared__ uint32_t s_q0;
    __shared__ uint64_t s_x0;
    const uint32_t n = a.m.n, t = threadIdx.x, lane = lane_id(), wave = t / kWave;
    const SumPair tail = a.sc[n];
    const uint64_t T = a.threshold;
    const uint32_t ncand = (uint32_t)tail.c;
    if (t == 0) {
        // the first span: pairs per file at the mean candidate size
        const double est = tail.s ? (double)T * (double)tail.c / (double)tail.s : 0.0;
        const uint32_t span = est < 1.0 ? 1u : est > (double)ncand ? ncand : (uint32_t)est;
        // the plateau path packs a flag into bit 31 of a position
        const uint32_t stop = n == 0 ? 1u : n >= 0x80000000u ? 2u : 0u;
        st = WalkState{0, 0, 0, span, kWalkMaxR, stop, 0, 0, 0};
    }
    __syncthreads();
    // phase 1: the one-shot prediction (merge_walk_abs_kernel's maps), chained
    // from file 0 in LDS; the files it resolves are written in parallel
    if (st.stop == 0 && a.abs_head[0] > 0) {
        const uint32_t nwin = a.abs_head[0];
        uint8_t *tab = lds_raw;
        for (uint32_t i = t; i < nwin * kAbsW / 8; i += kWalkThreads)
            reinterpret_cast<uint64_t *>(tab)[i] = reinterpret_cast<const uint64_t *>(a.abs_succ)[i];
        for (uint32_t i = t; i < 2 * nwin; i += kWalkThreads) s_bases[i] = a.abs_bases[i];
        const uint32_t x0 = a.abs_head[1];
        __syncthreads();
        if (t == 0) {
            uint32_t x = x0, f = 0;
            while (x < kAbsW) {  // file f ends at plateau base(f) + x
                s_chosen[f++] = (uint8_t)x;
                if (f == nwin || s_bases[2 * (f - 1) + 1] != s_bases[2 * f]) {
                    x = kAbsMiss;  // no map past the last window (or not the window it was mapped into)
                    break;
                }
                x = tab[(f - 1) * kAbsW + x];
            }
            s_nres = f;
            s_code = x;
        }
        __syncthreads();
        const uint32_t nres = s_nres, code = s_code;
        // thread f: file f's start (after file f - 1's end) and, for f < nres, its end
        uint64_t nw = 0, es = 0, Ps = 0;
        uint32_t pf = 0, wposf = kNone, wpermf = 0;
        if (t <= nres && t > 0) {
            es = s_bases[2 * (t - 1)] + s_chosen[t - 1];
            Ps = a.cand_pn[es - 1];
            uint64_t tg;
            walk_file(Ps, a.cand_pos[es - 1], a.cand_ext[es - 1], false, n, T, tail.s, pf, wposf, wpermf, tg);
        }
        if (t < nres) nw = (wposf != kNone ? 1 : 0) + (s_bases[2 * t] + s_chosen[t] - es);
        else if (t == nres && code == kAbsLast) nw = (wposf != kNone ? 1 : 0) + (tail.c - es);  // the rest fits
        uint64_t wt;
        const uint64_t wex = wave_excl_scan64(nw, &wt);
        const uint64_t wm = wave_max64(nw);
        if (lane == 0) {
            s_wsum[wave] = wt;
            s_wmax[wave] = wm;
        }
        __syncthreads();
        uint64_t pre = 0, tot = 0, most = 0;
        for (uint32_t w = 0; w < kWalkThreads / kWave; w++) {
            pre += w < wave ? s_wsum[w] : 0;
            tot += s_wsum[w];
            most = s_wmax[w] > most ? s_wmax[w] : most;
        }
        const uint64_t o = pre + wex;
        if (nw) {
            a.files[t] = MergeFile{pf, wposf, o};
            if (wposf != kNone) a.out[o] = wpermf;
        }
        if (t == nres && nres > 0) {  // the rounds go on from file nres's start
            WalkState x = st;
            x.p = pf;
            x.e = (uint32_t)es;
            x.P = Ps;
            x.nf = nres + (nw ? 1 : 0);
            x.o = tot;
            x.most = most;
            x.span = (uint32_t)((es + nres / 2) / nres);
            if (x.span == 0) x.span = 1;
            x.stop = code == kAbsLast || code == kAbsStop ? 1u : code == kAbsGeneral ? 2u : 0u;
            if (x.p >= n) x.stop = 1;
            st = x;
        } else if (t == 0 && nres == 0 && code == kAbsLast) {  // one file holds everything
            WalkState x = st;
            x.nf = nw ? 1 : 0;
            x.o = tot;
            x.most = most;
            x.stop = 1;
            st = x;
        }
        __syncthreads();
    }
    for (;;) {
        WalkState S0 = st;
        // every pass writes a file or hands the next one to the general step,
        // which writes one: more files than pairs cannot happen (fail-safe
        // against overrunning files[])
        if (S0.stop == 1 || S0.nf > n) break;
        __syncthreads();  // st is rewritten below
        if (S0.stop == 0 && S0.p != 0 && S0.e == 0) S0.stop = 2;  // no plateau before p
        if (S0.stop == 0) {
            const uint32_t R = S0.R, W = kWalkEntries / R;
            auto base = [&](uint32_t r) -> uint64_t {  // the first plateau of window r
                const uint64_t c = (uint64_t)S0.e + (uint64_t)(r + 1) * S0.span;
                return c > (uint64_t)S0.e + 1 + W / 2 ? c - W / 2 : (uint64_t)S0.e + 1;
            };
            for (uint32_t x = t; x < kWalkEntries; x += kWalkThreads) {
                const uint32_t r = x / W;
                const uint64_t e = base(r) + (x - r * W);
                uint64_t P = ~0ull, X = 0;
                uint32_t Q = 0;
                if (e <= ncand) {
                    P = a.cand_pn[e - 1];
                    Q = a.cand_pos[e - 1];
                    X = a.cand_ext[e - 1];
                }
                wp[x] = P;
                wq[x] = Q;
                wx[x] = X;
            }
            if (t == 0 && S0.p) {  // the round's first file starts after plateau S0.e
                s_q0 = a.cand_pos[S0.e - 1];
                s_x0 = a.cand_ext[S0.e - 1];
            }
            __syncthreads();
            // succession: plateau x of window r as the start of file r + 1;
            // a thread's plateaus search in lockstep (their LDS reads in
            // flight together)
            {
                constexpr uint32_t PT = kWalkEntries / kWalkThreads;
                uint64_t tg[PT];
                uint32_t b1[PT], pos[PT];
                uint16_t code[PT];
#pragma unroll
                for (uint32_t k = 0; k < PT; k++) {
                    const uint32_t x = t + k * kWalkThreads, r = x / W;
                    const uint64_t e = base(r) + (x - r * W);
                    code[k] = kSuccMiss;
                    tg[k] = ~0ull;
                    if (r + 1 < R && e <= ncand) {
                        uint32_t p, wpos, wperm;
                        code[k] = walk_file(wp[x], wq[x], wx[x], false, n, T, tail.s, p, wpos, wperm, tg[k]);
                    }
                    b1[k] = code[k] == 0 ? (r + 1) * W : 0;  // others search harmlessly
                    pos[k] = 0;
                }
                for (uint32_t s = W / 2; s > 0; s >>= 1) {
#pragma unroll
                    for (uint32_t k = 0; k < PT; k++)
                        if (wp[b1[k] + pos[k] + s - 1] < tg[k]) pos[k] += s;
                }
#pragma unroll
                for (uint32_t k = 0; k < PT; k++) {
                    const uint32_t x = t + k * kWalkThreads, r = x / W;
                    if (r + 1 >= R) continue;
                    if (code[k] == 0) {
                        const uint32_t lo = pos[k] + (wp[b1[k] + pos[k]] < tg[k] ? 1u : 0u);
                        const uint64_t e = base(r) + (x - r * W);
                        code[k] = (lo < W && (lo > 0 || base(r + 1) <= e + 1)) ? (uint16_t)lo : kSuccMiss;
                    }
                    sx[x] = code[k];
                }
            }
            __syncthreads();
            if (wave == 0) {
                // the round's first file starts after plateau S0.e (the state)
                const uint32_t Qs = S0.p ? s_q0 : 0;
                const uint64_t Xs = S0.p ? s_x0 : 0;
                uint32_t p, wpos, wperm;
                uint64_t tg;
                uint16_t code = walk_file(S0.P, Qs, Xs, S0.p == 0, n, T, tail.s, p, wpos, wperm, tg);
                if (p != S0.p) code = kSuccGeneral;  // not a plateau start (after an extra that filled a file)
                if (code == 0) {  // file 0's end: the first window-0 plateau at the target
                    code = kSuccMiss;
                    for (uint32_t i0 = 0; i0 < W; i0 += kWave) {
                        const uint64_t ge = __ballot(wp[i0 + lane] >= tg);
                        if (!ge) continue;
                        const uint32_t x = i0 + (uint32_t)__builtin_ctzll(ge);
                        if (x > 0 || base(0) <= (uint64_t)S0.e + 1) code = (uint16_t)x;
                        break;
                    }
                }
                // chain: file r ends at plateau x_r of window r (lane r keeps
                // it) while the files resolve; one LDS read per file
                uint32_t nres = 0, my_x = 0;
                while (code < kSuccLast) {
                    if (lane == nres) my_x = code;
                    nres++;
                    if (nres == R) break;
                    code = sx[(nres - 1) * W + code];
                }
                // every lane r <= nres: file r's start (after file r - 1's
                // end, or the state's) and, for r < nres, its end
                const uint32_t px = __shfl_up(my_x, 1);
                uint64_t Ps = S0.P, es = S0.e;
                uint32_t Qr = Qs;
                uint64_t Xr = Xs;
                if (lane > 0 && lane <= nres) {
                    const uint32_t y = (lane - 1) * W + px;
                    Ps = wp[y];
                    Qr = wq[y];
                    Xr = wx[y];
                    es = base(lane - 1) + px;
                }
                uint32_t pr = 0, wposr = kNone, wpermr = 0;
                uint64_t tgr;
                walk_file(Ps, Qr, Xr, lane == 0 && S0.p == 0, n, T, tail.s, pr, wposr, wpermr, tgr);
                if (lane == 0) pr = S0.p;
                uint64_t nw = 0;
                if (lane < nres) {
                    nw = (wposr != kNone ? 1 : 0) + (base(lane) + my_x - es);
                } else if (lane == nres && nres < R && code == kSuccLast) {
                    nw = (wposr != kNone ? 1 : 0) + (tail.c - es);  // the rest fits (merge.go:125-128)
                }
                uint64_t tot;
                const uint64_t ox = S0.o + wave_excl_scan64(nw, &tot);
                const uint64_t most = wave_max64(nw > S0.most ? nw : S0.most);
                if (nw) {
                    a.files[S0.nf + lane] = MergeFile{pr, wposr, ox};
                    if (wposr != kNone) a.out[ox] = wpermr;
                }
                // the next state: the start of file nres
                const uint32_t np = (uint32_t)__builtin_amdgcn_readlane((int)pr, (int)nres);
                const uint64_t ne = readlane64(es, nres), nP = readlane64(Ps, nres);
                uint32_t stop = 0, Rn = R;
                if (nres == R) {
                    Rn = R < kWalkMaxR ? 2 * R : R;  // every file of the round resolved
                    stop = np >= n ? 1u : 0u;
                } else if (code == kSuccStop || code == kSuccLast) {
                    stop = 1;
                } else if (code == kSuccGeneral) {
                    stop = 2;
                } else {  // kSuccMiss: the end lies outside the window: fewer files, wider windows
                    Rn = 1;
                    while (2 * Rn <= nres) Rn *= 2;
                    stop = nres == 0 ? 2u : 0u;  // nothing resolved: the general step
                }
                // files written: lanes 0 .. nres - 1, and lane nres for a last file
                const uint32_t nfn = S0.nf + (uint32_t)__builtin_popcountll(__ballot(nw != 0));
                uint32_t span = S0.span;
                if (nres > 0 && ne > S0.e) span = (uint32_t)((ne - S0.e + nres / 2) / nres);
                if (span == 0) span = 1;
                if (lane == 0) st = WalkState{np, (uint32_t)ne, nfn, span, Rn, stop, S0.o + tot, most, nP};
            }
            __syncthreads();
            continue;
        }
        // general step: the file starting at S0.p, by the whole workgroup
        const uint32_t p = S0.p;
        const bool starts = p == 0 || (a.flags[p] & 1);
        uint32_t g = p, w = kNone;
        uint64_t wsize = 0;
        if (!starts) {
            // the rest of the group: its end g and its first writable pair w
            for (uint32_t q0 = p;; q0 += kWalkThreads) {
                if (t < 2) s_min[t] = kNone;
                __syncthreads();
                const uint32_t qq = q0 + t;
                const uint8_t f = qq < n ? a.flags[qq] : 1;
                const bool endg = qq >= n || (qq > p && (f & 1));
                if (endg) atomicMin(&s_min[0], qq < n ? qq : n);
                __syncthreads();
                const uint32_t ge = s_min[0];
                if (!endg && qq < ge && (f & 2)) atomicMin(&s_min[1], qq);
                __syncthreads();
                if (w == kNone && s_min[1] != kNone) w = s_min[1];
                const bool fin = ge != kNone;
                if (fin) g = ge;
                __syncthreads();
                if (fin) break;
            }
            if (w != kNone) {
                const View v = view(a.m, a.perm[w]);
                wsize = 16 + (uint64_t)v.kl + v.vl;
            }
        }
        const uint64_t Sg = g < n ? a.sc[g].s : tail.s, Cg = g < n ? a.sc[g].c : tail.c;
        uint32_t end = n;
        if (w != kNone && wsize >= T) {
            end = w + 1;  // the extra alone fills the file
        } else {
            const uint64_t tg = Sg + (T - wsize);
            if (tail.s >= tg) {
                // first k in [g + 1, n] with S(k) >= tg: 1,024-way search rounds
                uint32_t lo = g + 1, hi = n;
                while (hi > lo) {
                    const uint32_t span = hi - lo;
                    const uint32_t step = span >= kWalkThreads - 1 ? (span + kWalkThreads - 2) / (kWalkThreads - 1) : 1;
                    uint32_t k = lo + t * step;
                    if (k > hi || t == kWalkThreads - 1) k = hi;
                    if (t == 0) s_min[0] = kNone;
                    __syncthreads();
                    const uint64_t sk = k < n ? a.sc[k].s : tail.s;
                    if (sk >= tg) atomicMin(&s_min[0], t);
                    __syncthreads();
                    const uint32_t f = s_min[0];
                    __syncthreads();
                    if (f == 0) { hi = lo; break; }
                    uint32_t kf = lo + f * step;
                    if (kf > hi || f == kWalkThreads - 1) kf = hi;
                    lo = lo + (f - 1) * step + 1;
                    hi = kf;
                }
                end = lo;  // the first position at or above the target; e = end - 1
            }
        }
        const SumPair Se = end < n ? a.sc[end] : tail;
        const uint64_t nw = (w != kNone ? 1 : 0) + (end > g ? Se.c - Cg : 0);
        if (t == 0) {
            WalkState x = S0;
            if (nw == 0) {
                x.stop = 1;  // nothing left to write: no file (builder.size == 0)
            } else {
                a.files[x.nf] = MergeFile{p, w, x.o};
                if (w != kNone) a.out[x.o] = a.perm[w];
                x.o += nw;
                x.most = nw > x.most ? nw : x.most;
                x.nf++;
                if (end > g && Se.c > Cg) x.span = (uint32_t)(Se.c - Cg);
                x.p = end;
                x.e = (uint32_t)Se.c;
                x.P = Se.s;
                // the plateau path again, unless positions exceed its packing
                x.stop = end >= n ? 1u : n >= 0x80000000u ? 2u : 0u;
            }
            st = x;
        }
        __syncthreads();
    }
    if (t == 0) {
        a.files[st.nf] = MergeFile{n, kNone, st.o};
        a.counts[0] = st.o;
        a.counts[1] = st.nf;
        a.counts[2] = st.most;
    }
}

// each candidate's output slot: its file's first slot, after the extra, plus
// the candidates before it in the file
__global__ __launch_bounds__(kMergeThreads) void merge_emit_kernel(
    const uint32_t *perm, const SumPair *sc, const uint32_t *csize, const MergeFile *files,
    const uint64_t *counts, uint32_t n, uint32_t *out, uint64_t *file_start, uint64_t *counts_out) {
    __shared__ uint32_t s_lo;
    const uint32_t j0 = blockIdx.x * kMergeThreads, j = j0 + threadIdx.x;
    const uint32_t nf = (uint32_t)counts[1];
    // the async form's device counts (no copy launch after this one)
    if (counts_out && j < 3) counts_out[j] = counts[j];
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

// The gather's key / value offsets: one scan of the selected pairs' (key
// length, value length) -- tile sums (the lengths kept), the tile sums'
// scan (merge_scan_partials), then each slot's offsets -- where two scans
// of separately gathered lengths took 88 us for 3.3M pairs.
// the gather's pair count: the host's, or lsm_gather_kvs_dev's device count,
// capped at the bound the grid and the klen / vlen / koff / voff arrays are
// sized from (a count above it is a caller error; the gather stays in bounds)
__device__ __forceinline__ uint32_t gather_count(uint32_t nmax, const uint64_t *d_nout) {
    if (!d_nout) return nmax;
    const uint64_t n = *d_nout;
    return n < nmax ? (uint32_t)n : nmax;
}

// The pass that reads every selected pair's descriptors (through idx, in
// output order) also leaves each key's source offset densely in output order
// (ksrc): the keys-only copy then reads no descriptor through idx (gather
// 0.145 -> 0.139-0.141 ms per compaction).  Leaving the values' views there
// too, for lsm_build_sst_views to read with no idx, cost the gather 26 us
// (54 MB more written) and saved the build 5 (A/B).
__global__ __launch_bounds__(kMergeThreads) void gather_scan_tiles(MergeIn m, const uint32_t *idx,
                                                                   uint32_t nmax, const uint64_t *d_nout,
                                                                   uint32_t *klen, uint32_t *vlen,
                                                                   SumPair *part, uint64_t *ksrc) {
    const uint32_t nout = gather_count(nmax, d_nout);
    uint64_t s = 0, c = 0;
    const uint64_t i0 = (uint64_t)blockIdx.x * kScanTile + threadIdx.x * kScanPer;
    for (uint32_t t = 0; t < kScanPer; t++) {
        if (i0 + t < nout) {
            const View v = view(m, idx[i0 + t]);
            klen[i0 + t] = v.kl;
            vlen[i0 + t] = v.vl;
            ksrc[i0 + t] = v.ko;
            s += v.kl;
            c += v.vl;
        }
    }
    SumPair tot;
    block_excl_scan2(s, c, &tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kMergeThreads) void gather_scan_apply(const uint32_t *klen,
                                                                   const uint32_t *vlen, uint32_t nmax,
                                                                   const uint64_t *d_nout,
                                                                   const SumPair *part,
                                                                   const SumPair *total, uint64_t *koff,
                                                                   uint64_t *voff) {
    const uint32_t nout = gather_count(nmax, d_nout);
    uint32_t kl[kScanPer], vl[kScanPer];
    uint64_t s = 0, c = 0;
    const uint64_t i0 = (uint64_t)blockIdx.x * kScanTile + threadIdx.x * kScanPer;
    for (uint32_t t = 0; t < kScanPer; t++) {
        kl[t] = i0 + t < nout ? klen[i0 + t] : 0;
        vl[t] = i0 + t < nout ? vlen[i0 + t] : 0;
        s += kl[t];
        c += vl[t];
    }
    SumPair tot;
    const SumPair x = block_excl_scan2(s, c, &tot);
    uint64_t ps = x.s + part[blockIdx.x].s, pc = x.c + part[blockIdx.x].c;
    for (uint32_t t = 0; t < kScanPer; t++) {
        if (i0 + t < nout) {
            koff[i0 + t] = ps;
            voff[i0 + t] = pc;
        }
        ps += kl[t];
        pc += vl[t];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        koff[nout] = total->s;
        voff[nout] = total->c;
    }
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
    MergeIn m, const uint32_t *idx, uint32_t nmax, const uint64_t *d_nout, const uint64_t *koff,
    const uint64_t *voff, uint8_t *keys, uint8_t *vals, const uint64_t *ksrc) {
    const uint32_t nout = gather_count(nmax, d_nout);
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
        const uint32_t j = j0 + lane;
        d0[0] = koff[j];
        d0[1] = voff[j];
        if (vals) {
            const View v = view(m, idx[j]);
            d1[0] = d0[0] + v.kl;
            d1[1] = d0[1] + v.vl;
            s_src[w][0][lane] = v.ko;
            s_src[w][1][lane] = v.vo;
        } else {  // keys only: the sources the scan left in output order
            d1[0] = koff[j + 1];
            d1[1] = voff[j + 1];
            s_src[w][0][lane] = ksrc[j];
        }
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
    uint64_t *xinfo;  // n: merge_flags_kernel's per-pair words for the walk's extras
    uint8_t *abs_succ;    // the walk's one-shot prediction (merge_walk_abs_kernel)
    uint64_t *abs_bases;
    uint32_t *abs_head;
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
    w.xinfo = reinterpret_cast<uint64_t *>(take(8 * nn));
    w.abs_succ = take((size_t)kAbsMaxWin * kAbsW);
    w.abs_bases = reinterpret_cast<uint64_t *>(take(16 * (size_t)kAbsMaxWin));
    w.abs_head = reinterpret_cast<uint32_t *>(take(8));
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
//
// Pop's down() is run bottom-up (Floyd): the hole left by the root goes down
// the path of smaller children -- the left one on ties, as down() picks --
// branch-free, to a leaf, and then the moved element rises while its parent's
// rank is >= its own.  down() moves up exactly the path elements whose rank
// is < the element's (it stops at the first child that is not less), and the
// path's ranks never decrease, so the rise puts back exactly the others: the
// same array as down() leaves, after every pop.  down()'s child choice is an
// unpredictable branch per level; here the descent has none, and it prefetches
// three and four levels ahead (a 64-byte block each).
void goheap_pop_order(const uint32_t *rank, uint32_t n, uint32_t *order, uint64_t *phase_ns = nullptr) {
    std::vector<uint64_t> h(n ? n : 1);
    uint64_t *H = h.data();
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 0; i < n; i++) {  // Push: append, up(h, i)
        const uint64_t x = (uint64_t)rank[i] << 32 | i;
        uint32_t j = i;
        while (j > 0) {
            const uint32_t p = (j - 1) / 2;
            if (!((x >> 32) < (H[p] >> 32))) break;
            H[j] = H[p];
            j = p;
        }
        H[j] = x;
    }
    const auto t1 = std::chrono::steady_clock::now();
    for (uint32_t r = n; r > 0; r--) {  // Pop: swap(0, r-1), down(0, r-1)
        const uint64_t top = H[0], x = H[r - 1];
        const uint32_t m = r - 1, xr = (uint32_t)(x >> 32);
        uint32_t i = 0;
        while (2 * i + 2 < m) {  // both children in the heap
            const uint32_t j1 = 2 * i + 1;
            __builtin_prefetch(&H[8 * (uint64_t)i + 7]);
            __builtin_prefetch(&H[16 * (uint64_t)i + 15]);
            const uint64_t a = H[j1], b = H[j1 + 1];
            const uint32_t j = j1 + (uint32_t)((b >> 32) < (a >> 32));  // the right one only if less
            H[i] = H[j];
            i = j;
        }
        if (2 * i + 1 < m) {  // a left child only
            H[i] = H[2 * i + 1];
            i = 2 * i + 1;
        }
        while (i > 0) {  // back up past every path element whose rank is >= x's
            const uint32_t p = (i - 1) / 2;
            if ((uint32_t)(H[p] >> 32) < xr) break;
            H[i] = H[p];
            i = p;
        }
        if (m) H[i] = x;
        H[m] = top;
        order[n - r] = (uint32_t)top;
    }
    if (phase_ns) {
        const auto t2 = std::chrono::steady_clock::now();
        phase_ns[0] = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
        phase_ns[1] = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t2 - t1).count();
    }
}

}  // namespace lsm

using namespace lsm;

extern "C" int lsm_goheap_pop_order_host(const uint32_t *rank, uint64_t n, uint32_t *order,
                                         uint64_t *phase_ns) {
    if (n >= 0xFFFFFFFFull || (n && (!rank || !order))) return LSM_EINVAL;
    goheap_pop_order(rank, (uint32_t)n, order, phase_ns);
    return 0;
}

extern "C" uint64_t lsm_goheap_replays(const lsm_ctx *ctx) { return ctx ? ctx->goheap_replays : 0; }

static_assert(sizeof(MergeFile) == 16, "MergeFile layout");
static_assert(sizeof(SumPair) == 16, "SumPair layout");

extern "C" size_t lsm_merge_kvs_workspace_bytes(uint64_t n) {
    if (n >= 0xFFFFFFFFull) return 0;
    return merge_ws_layout(nullptr, (uint32_t)n).total;
}

namespace lsm {
namespace {

// The others as a k-way merge.  The pairs outside the longest run are, in
// input order, a few sorted runs when the input is a compaction's files (each
// file is sorted: level 0's flushes and the pieces of level 1 around the run),
// and the key statistics count the input's descents exactly, which bounds the
// runs.  With at most kKwayMaxRuns runs the others are ranked instead of
// radix-sorted: a pair's place is its place in its own run plus, in every
// other run, the pairs before it -- those <= its key in an earlier run, < in a
// later one (the stable order: equal keys in input order, as the radix sort
// leaves them).  merge_kway_runs_kernel lists the run starts (a descent of
// the packed keys, or the junction of the pairs before the long run with those
// after it); merge_kway_rank_kernel sorts the list, stages every kKwaySample-th
// key of each run in LDS, and per pair searches all runs side by side: first
// in the samples, then in the one sample interval in global memory.
constexpr uint32_t kKwayMaxRuns = 12;
constexpr uint32_t kKwayThreads = 1024;
constexpr uint32_t kKwaySamples = 4096;  // LDS samples per workgroup, all runs

template <class K>
__global__ __launch_bounds__(kMergeThreads) void merge_kway_runs_kernel(const K *ok0, uint32_t no, uint32_t junction,
                                                                        uint32_t *list) {
    // list[0] (the count) was zeroed by merge_extract_split_kernel
    const uint32_t j = blockIdx.x * kMergeThreads + threadIdx.x + 1;
    if (j < no && (j == junction || ok0[j] < ok0[j - 1])) {
        const uint32_t q = atomicAdd(&list[0], 1u);
        if (q < 2 * kKwayMaxRuns) list[1 + q] = j;
    }
}

template <class K>
__global__ __launch_bounds__(kKwayThreads) void merge_kway_rank_kernel(const K *ok0, const uint32_t *oi0, uint32_t no,
                                                                       const uint32_t *list, K *ok1, uint32_t *oi1) {
    __shared__ uint32_t sb[kKwayMaxRuns + 1];  // run b = [sb[b], sb[b + 1])
    __shared__ uint32_t sbase[kKwayMaxRuns + 1];  // its first sample
    __shared__ uint32_t s_R, s_stride;
    __shared__ K smp[kKwaySamples + kKwayMaxRuns];
    if (threadIdx.x == 0) {
        // the host's bound admits at most kKwayMaxRuns - 1 starts past 0
        uint32_t p[kKwayMaxRuns];
        const uint32_t c = list[0], n = c < kKwayMaxRuns - 1 ? c : kKwayMaxRuns - 1;
        for (uint32_t a = 0; a < n; a++) {  // insertion sort of the starts
            const uint32_t x = list[1 + a];
            uint32_t b = a;
            while (b > 0 && p[b - 1] > x) {
                p[b] = p[b - 1];
                b--;
            }
            p[b] = x;
        }
        sb[0] = 0;
        for (uint32_t a = 0; a < n; a++) sb[a + 1] = p[a];
        sb[n + 1] = no;
        s_R = n + 1;
        // every stride-th key of a run, so that all runs' samples fit
        const uint32_t st = (no + kKwaySamples - 1) / kKwaySamples;
        s_stride = st < 1 ? 1 : st;
        uint32_t o = 0;
        for (uint32_t b = 0; b <= n; b++) {
            sbase[b] = o;
            o += (sb[b + 1] - sb[b] + s_stride - 1) / s_stride;
        }
        sbase[n + 1] = o;
    }
    __syncthreads();
    const uint32_t R = s_R, stride = s_stride;
    for (uint32_t b = 0; b < R; b++) {
        const uint32_t cnt = sbase[b + 1] - sbase[b];
        for (uint32_t t = threadIdx.x; t < cnt; t += kKwayThreads) smp[sbase[b] + t] = ok0[sb[b] + t * stride];
    }
    __syncthreads();
    const uint32_t j = blockIdx.x * kKwayThreads + threadIdx.x;
    if (j >= no) return;
    const K k = ok0[j];
    uint32_t a = 0;
    while (a + 1 < R && sb[a + 1] <= j) a++;
    // the bound in run b: the first position whose key is > k (earlier runs)
    // or >= k (later runs); samples first, then the one interval between two
    uint32_t lo[kKwayMaxRuns], hi[kKwayMaxRuns];
#pragma unroll
    for (uint32_t b = 0; b < kKwayMaxRuns; b++) {
        uint32_t l = 0, h = 0;
        if (b < R && b != a) {  // samples: the first sample index t with smp > / >= k
            l = sbase[b];
            h = sbase[b + 1];
            while (l < h) {
                const uint32_t mid = (l + h) >> 1;
                const K x = smp[mid];
                if (b < a ? x <= k : x < k) l = mid + 1;
                else h = mid;
            }
            // positions before sample t are all "before"; the bound is in
            // (position of sample t - 1, position of sample t]
            const uint32_t t = l - sbase[b];
            const uint32_t end = sb[b + 1];
            lo[b] = t == 0 ? sb[b] : sb[b] + (t - 1) * stride + 1;
            hi[b] = sb[b] + t * stride < end ? sb[b] + t * stride : end;
        } else {
            lo[b] = hi[b] = 0;
        }
    }
    for (;;) {
        bool any = false;
        K x[kKwayMaxRuns];
#pragma unroll
        for (uint32_t b = 0; b < kKwayMaxRuns; b++)
            if (lo[b] < hi[b]) x[b] = ok0[(lo[b] + hi[b]) >> 1];
#pragma unroll
        for (uint32_t b = 0; b < kKwayMaxRuns; b++) {
            if (lo[b] < hi[b]) {
                const uint32_t mid = (lo[b] + hi[b]) >> 1;
                if (b < a ? x[b] <= k : x[b] < k) lo[b] = mid + 1;
                else hi[b] = mid;
                any = true;
            }
        }
        if (!any) break;
    }
    uint32_t pos = j - sb[a];
#pragma unroll
    for (uint32_t b = 0; b < kKwayMaxRuns; b++)
        if (b < R && b != a) pos += lo[b] - sb[b];
    ok1[pos] = k;
    oi1[pos] = oi0[j];
}

}  // namespace
}  // namespace lsm

// The merge path (merge_rank_*): the pairs outside the run [rs, re) are
// packed and sorted (with their input index: ranked as a k-way merge when
// they are at most kKwayMaxRuns sorted runs, radix-sorted otherwise), the
// run's keys packed, and each pair's sorted position written to w.perm[0].
// Workspace: the run's keys in w.keys[0]; the others' keys (two buffers) in
// w.keys[1] and their indices in w.perm[1] (no <= n / 2).
template <class K>
static int merge_path(const MergeWs &w, const MergeIn &m, const SortGroup &g, uint32_t bits,
                      uint32_t rs, uint32_t re, uint32_t no, uint64_t descents, hipStream_t s) {
    const uint32_t N = m.n, nrun = re - rs;
    K *run_keys = reinterpret_cast<K *>(w.keys[0]);
    K *ok0 = reinterpret_cast<K *>(w.keys[1]), *ok1 = ok0 + no;
    uint32_t *oi0 = w.perm[1], *oi1 = w.perm[1] + no;
    const bool kway = no && descents + 2 <= kKwayMaxRuns && w.sort_bytes >= 4 * (2 * kKwayMaxRuns + 1);
    uint32_t *list = kway ? static_cast<uint32_t *>(w.sort_tmp) : nullptr;
    hipLaunchKernelGGL(merge_extract_split_kernel<K>, dim3(grid_for(N)), dim3(kMergeThreads), 0, s, m,
                       g, rs, re, run_keys, ok0, oi0, list);
    if (kway) {
        // the others' runs: the input's descents outside [rs, re), and the
        // junction of the pairs before the run with those after it
        hipLaunchKernelGGL(merge_kway_runs_kernel<K>, dim3(grid_for(no)), dim3(kMergeThreads), 0, s, ok0, no,
                           rs, list);
        hipLaunchKernelGGL(merge_kway_rank_kernel<K>, dim3((no + kKwayThreads - 1) / kKwayThreads),
                           dim3(kKwayThreads), 0, s, ok0, oi0, no, list, ok1, oi1);
        hipLaunchKernelGGL(merge_rank_others_kernel<K>, dim3(grid_for(no)), dim3(kMergeThreads), 0, s,
                           run_keys, nrun, rs, ok1, oi1, no, w.perm[0]);
    } else if (no) {
        size_t tb = w.sort_bytes;
        const hipError_t e = rocprim::radix_sort_pairs(w.sort_tmp, tb, ok0, ok1, oi0, oi1, no, 0, bits, s);
        if (e != hipSuccess) return -(1000 + (int)e);
        hipLaunchKernelGGL(merge_rank_others_kernel<K>, dim3(grid_for(no)), dim3(kMergeThreads), 0, s,
                           run_keys, nrun, rs, ok1, oi1, no, w.perm[0]);
    }
    hipLaunchKernelGGL(merge_rank_run_kernel<K>, dim3(grid_for(nrun)), dim3(kMergeThreads), 0, s,
                       run_keys, nrun, rs, ok1, oi1, no, w.perm[0]);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}

// h_counts (host, read back) or d_counts (device, left there: the async form)
static int merge_kvs(lsm_ctx *ctx, const uint8_t *d_bytes, const lsm_rec_desc *d_key_desc,
                     const lsm_rec_desc *d_val_desc, uint64_t n, int level, uint64_t threshold,
                     int tie, uint32_t *d_out, uint64_t *d_file_start, uint64_t *h_counts,
                     uint64_t *d_counts, void *d_ws, size_t ws_bytes, void *stream,
                     const uint64_t *d_expect_n = nullptr) {
    if (!ctx || (!h_counts && !d_counts) || threshold == 0 || n >= 0xFFFFFFFFull) return LSM_EINVAL;
    if (tie != LSM_TIE_INPUT && tie != LSM_TIE_GOHEAP) return LSM_EINVAL;
    if (n && (!d_bytes || !d_key_desc || !d_out || !d_ws)) return LSM_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (h_counts) h_counts[0] = h_counts[1] = h_counts[2] = 0;
    // d_expect_n (lsm_compact_merge_async): the join's pair count, computed on
    // the device, read back with the key statistics and checked against n
    uint64_t *expect_h = reinterpret_cast<uint64_t *>(static_cast<uint8_t *>(ctx->host_rb) + kHostReadback - 64);
    if (n == 0 && d_expect_n) {
        LSM_HIP_CHECK(hipMemcpyAsync(expect_h, d_expect_n, 8, hipMemcpyDeviceToHost, s));
        LSM_HIP_CHECK(hipStreamSynchronize(s));
        if (*expect_h != 0) return LSM_EINVAL;
    }
    if (n == 0) {
        if (d_file_start) LSM_HIP_CHECK(hipMemsetAsync(d_file_start, 0, 8, s));
        if (d_counts) LSM_HIP_CHECK(hipMemsetAsync(d_counts, 0, 24, s));
        return 0;
    }
    const uint32_t N = (uint32_t)n;
    MergeWs w = merge_ws_layout(static_cast<uint8_t *>(d_ws), N);
    if (ws_bytes < w.total) return LSM_ESPACE;
    const MergeIn m{d_bytes, d_key_desc, d_val_desc, N};
    const uint32_t sb = grid_for(n) < kStatBlocks ? grid_for(n) : kStatBlocks;

    // 1. key statistics and the sorted runs: one pass over contiguous
    //    tiles, per-tile partials reduced here
    const uint32_t chunk = (N + sb - 1) / sb;
    hipLaunchKernelGGL(merge_stats_kernel, dim3(sb), dim3(kMergeThreads), 0, s, m, chunk, w.part);
    static_assert((size_t)kStatBlocks * kStatWords * 8 + 64 <= kHostReadback - 64, "read-back buffer");
    const uint64_t *part = static_cast<const uint64_t *>(ctx->host_rb);  // pinned
    LSM_HIP_CHECK(hipMemcpyAsync(ctx->host_rb, w.part, (size_t)sb * kStatWords * 8, hipMemcpyDeviceToHost, s));
    if (d_expect_n) LSM_HIP_CHECK(hipMemcpyAsync(expect_h, d_expect_n, 8, hipMemcpyDeviceToHost, s));
    LSM_HIP_CHECK(hipStreamSynchronize(s));
    if (d_expect_n && *expect_h != n) return LSM_EINVAL;  // n is not the join's pair count
    uint64_t st[kStatCore];
    for (uint32_t t = 0; t < kStatCore; t++) st[t] = part[t];
    uint64_t run_s = 0, run_e = 0, cur_s = 0;  // the longest run found, the open one
    uint64_t descents = 0;                     // of the whole input (exact)
    auto run = [&](uint64_t a, uint64_t b) {
        if (b - a > run_e - run_s) { run_s = a; run_e = b; }
    };
    for (uint32_t b = 0; b < sb; b++) {
        const uint64_t *q = &part[(size_t)b * kStatWords];
        if (b) {
            st[0] = q[0] > st[0] ? q[0] : st[0];
            st[1] = q[1] < st[1] ? q[1] : st[1];
            for (uint32_t t = 2; t < kStatCore; t += 2) {
                st[t] |= q[t];
                st[t + 1] &= q[t + 1];
            }
        }
        const uint64_t *r = q + kStatCore;  // first, last descent, count, inner run
        descents += r[2];
        if (r[2] == 0) continue;
        run(cur_s, r[0]);
        if (r[4] > r[3]) run(r[3], r[4]);
        cur_s = r[1];
    }
    run(cur_s, N);
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
    // the merge path: every varying bit in one packed key and one sorted run
    // holding at least half the pairs
    uint32_t all_bits = 0;
    for (const auto &f : fields) all_bits += (uint32_t)__builtin_popcountll(f.second);
    const uint32_t rs = (uint32_t)run_s, re = (uint32_t)run_e, no = N - (re - rs);
    if (!fields.empty() && fields.size() <= kGroupFields && all_bits <= 64 && no <= N / 2 &&
        N >= kMergePathMin) {
        SortGroup g{};
        g.nf = (uint32_t)fields.size();
        for (size_t t = 0; t < g.nf; t++) {  // most significant first
            g.field[t] = fields[g.nf - 1 - t].first;
            g.mask[t] = fields[g.nf - 1 - t].second;
        }
        const int rc = all_bits <= 32
                           ? merge_path<uint32_t>(w, m, g, all_bits, rs, re, no, descents, s)
                           : merge_path<uint64_t>(w, m, g, all_bits, rs, re, no, descents, s);
        if (rc) return rc;
        fields.clear();
        have_perm = true;  // w.perm[0]
    }
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
        // ranks by input index on the device (newgroup flags, tile scan,
        // scatter), read back into the context's pinned buffer; the order
        // goes back from the same buffer
        const uint32_t ntiles = (N + kScanTile - 1) / kScanTile;
        uint32_t *rank_d = w.perm[cur ^ 1];
        hipLaunchKernelGGL(goheap_newgroup_kernel, dim3(grid_for(n)), dim3(kMergeThreads), 0, s, m,
                           perm, w.csize);
        hipLaunchKernelGGL(merge_scan_tiles, dim3(ntiles), dim3(kMergeThreads), 0, s, w.csize, N,
                           w.scan_part);
        hipLaunchKernelGGL(merge_scan_partials, dim3(1), dim3(kPartThreads), 0, s, w.scan_part, ntiles,
                           w.sc, N);
        hipLaunchKernelGGL(goheap_rank_apply, dim3(ntiles), dim3(kMergeThreads), 0, s, w.csize, N,
                           w.scan_part, perm, rank_d);
        LSM_HIP_CHECK(hipGetLastError());
        // Every key distinct (N - 1 new-key flags: position 0 has rank 0 and
        // no flag): the heap pops in key order, the sorted order already is
        // its pop order -- no replay
        SumPair *ng = static_cast<SumPair *>(ctx->host_rb);  // pinned
        LSM_HIP_CHECK(hipMemcpyAsync(ng, w.sc + N, sizeof(SumPair), hipMemcpyDeviceToHost, s));
        LSM_HIP_CHECK(hipStreamSynchronize(s));
        ctx->goheap_replays += ng->s + 1 != N;
    }
    if (tie == LSM_TIE_GOHEAP && static_cast<SumPair *>(ctx->host_rb)->s + 1 != N) {
        uint32_t *rank_d = w.perm[cur ^ 1];
        const size_t need = 8ull * N;  // ranks, then the pop order
        if (ctx->host_big_bytes < need) {
            LSM_HIP_CHECK(hipStreamSynchronize(s));
            if (ctx->host_big) LSM_HIP_CHECK(hipHostFree(ctx->host_big));
            ctx->host_big = nullptr;
            ctx->host_big_bytes = 0;
            LSM_HIP_CHECK(hipHostMalloc(&ctx->host_big, need, hipHostMallocDefault));
            ctx->host_big_bytes = need;
        }
        uint32_t *hrank = static_cast<uint32_t *>(ctx->host_big), *horder = hrank + N;
        LSM_HIP_CHECK(hipMemcpyAsync(hrank, rank_d, 4ull * N, hipMemcpyDeviceToHost, s));
        LSM_HIP_CHECK(hipStreamSynchronize(s));
        goheap_pop_order(hrank, N, horder);
        LSM_HIP_CHECK(hipMemcpyAsync(w.perm[cur], horder, 4ull * N, hipMemcpyHostToDevice, s));
        LSM_HIP_CHECK(hipStreamSynchronize(s));  // the pinned buffer is reused by the next call
    }

    // 3. groups and candidates; 4. sums and the file walk; 5. emit
    hipLaunchKernelGGL(merge_flags_kernel, dim3(grid_for(n)), dim3(kMergeThreads), 0, s, m, perm,
                       level, w.flags, w.csize, w.xinfo);
    hipLaunchKernelGGL(merge_candidate_kernel, dim3(grid_for(n)), dim3(kMergeThreads), 0, s, m,
                       w.flags, w.csize);
    const uint32_t ntiles = (N + kScanTile - 1) / kScanTile;
    hipLaunchKernelGGL(merge_scan_tiles, dim3(ntiles), dim3(kMergeThreads), 0, s, w.csize, N,
                       w.scan_part);
    hipLaunchKernelGGL(merge_scan_partials, dim3(1), dim3(kPartThreads), 0, s, w.scan_part, ntiles,
                       w.sc, N);
    // the walk's plateau arrays in the sort's buffers, free from here on
    uint64_t *cand_pn = w.keys[0], *cand_ext = w.keys[1];
    uint32_t *cand_pos = w.perm[cur ^ 1];
    hipLaunchKernelGGL(merge_scan_apply, dim3(ntiles), dim3(kMergeThreads), 0, s, w.csize, N,
                       w.scan_part, w.sc, w.flags, m, perm, w.xinfo, cand_pn, cand_pos, cand_ext);
    const AbsArgs aa{cand_pn, cand_pos, cand_ext, w.sc, N, threshold, w.abs_succ, w.abs_bases, w.abs_head};
    hipLaunchKernelGGL(merge_walk_abs_kernel, dim3(kAbsMaxWin), dim3(kAbsThreads), 0, s, aa);
    WalkArgs wa{m, perm, w.flags, w.sc, cand_pn, cand_pos, cand_ext, w.abs_succ, w.abs_bases, w.abs_head,
                threshold, w.files, d_out, w.stats};
    hipLaunchKernelGGL(merge_walk_kernel, dim3(1), dim3(kWalkThreads), 0, s, wa);
    hipLaunchKernelGGL(merge_emit_kernel, dim3(grid_for(n + 1)), dim3(kMergeThreads), 0, s, perm,
                       w.sc, w.csize, w.files, w.stats, N, d_out, d_file_start, d_counts);
    LSM_HIP_CHECK(hipGetLastError());
    if (d_counts) return 0;  // the async form: the counts stay on the device (written by the emit)
    uint64_t *c3 = static_cast<uint64_t *>(ctx->host_rb);  // pinned
    LSM_HIP_CHECK(hipMemcpyAsync(c3, w.stats, 3 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    LSM_HIP_CHECK(hipStreamSynchronize(s));
    for (int i = 0; i < 3; i++) h_counts[i] = c3[i];
    return 0;
}

extern "C" int lsm_merge_kvs_tie(lsm_ctx *ctx, const uint8_t *d_bytes,
                                 const lsm_rec_desc *d_key_desc, const lsm_rec_desc *d_val_desc,
                                 uint64_t n, int level, uint64_t threshold, int tie,
                                 uint32_t *d_out, uint64_t *d_file_start, uint64_t *h_counts,
                                 void *d_ws, size_t ws_bytes, void *stream) {
    if (!h_counts) return LSM_EINVAL;
    return merge_kvs(ctx, d_bytes, d_key_desc, d_val_desc, n, level, threshold, tie, d_out,
                     d_file_start, h_counts, nullptr, d_ws, ws_bytes, stream);
}

extern "C" int lsm_merge_kvs_async(lsm_ctx *ctx, const uint8_t *d_bytes,
                                   const lsm_rec_desc *d_key_desc, const lsm_rec_desc *d_val_desc,
                                   uint64_t n, int level, uint64_t threshold, int tie,
                                   uint32_t *d_out, uint64_t *d_file_start, uint64_t *d_counts,
                                   void *d_ws, size_t ws_bytes, void *stream) {
    if (!d_counts) return LSM_EINVAL;
    return merge_kvs(ctx, d_bytes, d_key_desc, d_val_desc, n, level, threshold, tie, d_out,
                     d_file_start, nullptr, d_counts, d_ws, ws_bytes, stream);
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
    return 2 * ((4 * nn + 255) & ~(size_t)255) + ((8 * nn + 255) & ~(size_t)255) +
           sizeof(SumPair) * (ntiles + 1) + 256;
}

static int gather_kvs(lsm_ctx *ctx, const uint8_t *d_bytes, const lsm_rec_desc *d_key_desc,
                      const lsm_rec_desc *d_val_desc, const uint32_t *d_idx, uint64_t nout,
                      const uint64_t *d_nout, uint8_t *d_keys, uint64_t *d_koff, uint8_t *d_vals,
                      uint64_t *d_voff, void *d_ws, size_t ws_bytes, void *stream) {
    if (!ctx || !d_koff || !d_voff || nout >= 0xFFFFFFFFull) return LSM_EINVAL;
    if (nout && (!d_bytes || !d_key_desc || !d_idx || !d_keys || !d_ws)) return LSM_EINVAL;
    if (ws_bytes < lsm_gather_kvs_workspace_bytes(nout)) return LSM_ESPACE;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint32_t N = (uint32_t)nout;  // the count, or (device count) its bound
    const size_t nn = nout ? nout : 1, part = (4 * nn + 255) & ~(size_t)255;
    uint32_t *kl = static_cast<uint32_t *>(d_ws);
    uint32_t *vl = reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(d_ws) + part);
    uint64_t *ksrc = reinterpret_cast<uint64_t *>(static_cast<uint8_t *>(d_ws) + 2 * part);
    SumPair *tparts = reinterpret_cast<SumPair *>(static_cast<uint8_t *>(d_ws) + 2 * part +
                                                  ((8 * nn + 255) & ~(size_t)255));
    const uint32_t ntiles = (uint32_t)((nn + kScanTile - 1) / kScanTile);
    SumPair *total = tparts + ntiles;
    const MergeIn m{d_bytes, d_key_desc, d_val_desc, N};
    if (N == 0) {  // (a device count is then 0 as well)
        LSM_HIP_CHECK(hipMemsetAsync(d_koff, 0, 8, s));
        LSM_HIP_CHECK(hipMemsetAsync(d_voff, 0, 8, s));
        return 0;
    }
    hipLaunchKernelGGL(gather_scan_tiles, dim3(ntiles), dim3(kMergeThreads), 0, s, m, d_idx, N, d_nout,
                       kl, vl, tparts, ksrc);
    hipLaunchKernelGGL(merge_scan_partials, dim3(1), dim3(kPartThreads), 0, s, tparts, ntiles, total, 0);
    hipLaunchKernelGGL(gather_scan_apply, dim3(ntiles), dim3(kMergeThreads), 0, s, kl, vl, N, d_nout,
                       tparts, total, d_koff, d_voff);
    hipLaunchKernelGGL(gather_copy_kernel, dim3((N + kMergeThreads - 1) / kMergeThreads),
                       dim3(kMergeThreads), 0, s, m, d_idx, N, d_nout, d_koff, d_voff, d_keys, d_vals,
                       ksrc);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}

extern "C" int lsm_gather_kvs(lsm_ctx *ctx, const uint8_t *d_bytes, const lsm_rec_desc *d_key_desc,
                              const lsm_rec_desc *d_val_desc, const uint32_t *d_idx, uint64_t nout,
                              uint8_t *d_keys, uint64_t *d_koff, uint8_t *d_vals, uint64_t *d_voff,
                              void *d_ws, size_t ws_bytes, void *stream) {
    return gather_kvs(ctx, d_bytes, d_key_desc, d_val_desc, d_idx, nout, nullptr, d_keys, d_koff,
                      d_vals, d_voff, d_ws, ws_bytes, stream);
}

extern "C" int lsm_gather_kvs_dev(lsm_ctx *ctx, const uint8_t *d_bytes, const lsm_rec_desc *d_key_desc,
                                  const lsm_rec_desc *d_val_desc, const uint32_t *d_idx,
                                  const uint64_t *d_nout, uint64_t nout_max, uint8_t *d_keys,
                                  uint64_t *d_koff, uint8_t *d_vals, uint64_t *d_voff, void *d_ws,
                                  size_t ws_bytes, void *stream) {
    if (!d_nout) return LSM_EINVAL;
    return gather_kvs(ctx, d_bytes, d_key_desc, d_val_desc, d_idx, nout_max, d_nout, d_keys, d_koff,
                      d_vals, d_voff, d_ws, ws_bytes, stream);
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

// loadLevelData's join (lsm_sst_pairs) and CompactAndMergeKVs
// (lsm_merge_kvs_async) as one entry, queued in that order on one stream.
// Computing the merge's key statistics from the decoded index descriptors
// before the join (so the statistics' read-back overlaps the join) was
// measured and dropped: 1.062-1.074 ms per compaction against 1.029-1.035 ms
// for the two calls in sequence (A/B, profiles/r05d_compact_join_ab.txt).
extern "C" int lsm_compact_merge_async(lsm_ctx *ctx, const uint8_t *d_img, const lsm_sst_meta *d_meta,
                                       const uint64_t *d_file_off, uint32_t nfile,
                                       const lsm_rec_desc *d_idx_desc, const lsm_rec_desc *d_data_desc,
                                       uint64_t n, lsm_rec_desc *d_key_out, lsm_rec_desc *d_val_out,
                                       uint64_t *d_prefix, int level, uint64_t threshold, int tie,
                                       uint32_t *d_out, uint64_t *d_file_start, uint64_t *d_counts,
                                       void *d_ws, size_t ws_bytes, void *stream) {
    if (!ctx || !d_prefix || !d_counts || threshold == 0 || n >= 0xFFFFFFFFull) return LSM_EINVAL;
    if (tie != LSM_TIE_INPUT && tie != LSM_TIE_GOHEAP) return LSM_EINVAL;
    const int rc = lsm_sst_pairs(ctx, d_meta, d_file_off, nfile, d_idx_desc, d_data_desc, d_key_out,
                                 d_val_out, d_prefix, stream);
    if (rc) return rc;
    return merge_kvs(ctx, d_img, d_key_out, d_val_out, n, level, threshold, tie, d_out, d_file_start,
                     nullptr, d_counts, d_ws, ws_bytes, stream, d_prefix + nfile);
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
