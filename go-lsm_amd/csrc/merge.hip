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
// wins -- and merge_test.go:25,53 checks it; this path implements that
// contract: equal keys leave in input order.
//
// GPU shape:
//   1. key statistics (max / min key length; per 8-byte chunk the OR and AND
//      of every key's big-endian chunk) -> the host picks the radix passes;
//   2. LSD radix passes (rocPRIM onesweep, stable) on the key length, then
//      chunk D-1 .. chunk 0 (zero padded), each over only the bits that vary:
//      the result is Go string order with input order on full ties;
//   3. group flags (a key differing from its predecessor starts a group; an
//      empty key is its own group because "" is never deduplicated) and the
//      candidate of each group: its first pair that may be written;
//   4. scans of the candidates' sizes and counts, then one wave walks the
//      file boundaries (a flush inside a group makes the next writable pair
//      of that group a write of its own -- the "extra" of the next file);
//   5. emit: each candidate's output slot from its file's start.
// Steps 3-5 are exact for any input; only the tie order is specified above.

#include <rocprim/device/device_radix_sort.hpp>

#include <vector>

#include "common.h"

namespace lsm {

int scan_u32_to_u64(const uint32_t *d_len, uint32_t n, uint64_t *d_out, void *ws, size_t ws_bytes,
                    hipStream_t s);
size_t scan_workspace_bytes(uint32_t n);

namespace {

constexpr uint32_t kMergeThreads = 256;
constexpr uint32_t kStatBlocks = 1024;
constexpr uint32_t kMaxChunks = kKeyCap / 8 + 1;  // 1 MiB keys
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint64_t kFileBytes = 16;  // MergeFile

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

__device__ __forceinline__ uint32_t key_len(const MergeIn &m, uint32_t i) {
    return reinterpret_cast<const uint32_t *>(m.kd + i)[2];
}

// Big-endian 8-byte chunk d of the key, zero past its end.
__device__ __forceinline__ uint64_t key_chunk(const uint8_t *p, uint32_t kl, uint32_t d) {
    uint64_t c = 0;
    const uint32_t b0 = 8 * d;
#pragma unroll
    for (uint32_t t = 0; t < 8; t++) {
        const uint8_t b = b0 + t < kl ? p[b0 + t] : 0;
        c = c << 8 | b;
    }
    return c;
}

__device__ __forceinline__ uint64_t wave_or64(uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ uint64_t wave_and64(uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) v &= __shfl_xor(v, o);
    return v;
}

// stats[0] = max key length, stats[1] = min key length (as u64 words)
__global__ __launch_bounds__(kMergeThreads) void merge_len_kernel(MergeIn m, uint64_t *stats) {
    uint32_t mx = 0, mn = 0xFFFFFFFFu;
    for (uint32_t i = blockIdx.x * kMergeThreads + threadIdx.x; i < m.n;
         i += gridDim.x * kMergeThreads) {
        const uint32_t kl = key_len(m, i);
        mx = kl > mx ? kl : mx;
        mn = kl < mn ? kl : mn;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t a = __shfl_xor(mx, o), b = __shfl_xor(mn, o);
        mx = a > mx ? a : mx;
        mn = b < mn ? b : mn;
    }
    if (lane_id() == 0) {
        atomicMax(reinterpret_cast<unsigned long long *>(&stats[0]), (unsigned long long)mx);
        atomicMin(reinterpret_cast<unsigned long long *>(&stats[1]), (unsigned long long)mn);
    }
}

// chunk statistics: orand[2d] = OR, orand[2d+1] = AND of chunk d over keys
// longer than 8d (shorter keys hold 0 there: the host folds that in with the
// minimum key length); orand[2D], [2D+1] = OR / AND of the key lengths
__global__ __launch_bounds__(kMergeThreads) void merge_chunk_stats_kernel(MergeIn m, uint32_t D,
                                                                          uint64_t *orand) {
    const uint32_t i0 = blockIdx.x * kMergeThreads + threadIdx.x, step = gridDim.x * kMergeThreads;
    uint64_t lo = 0, la = ~0ull;
    for (uint32_t i = i0; i < m.n; i += step) {
        const uint32_t kl = key_len(m, i);
        lo |= kl;
        la &= kl;
    }
    lo = wave_or64(lo);
    la = wave_and64(la);
    if (lane_id() == 0) {
        atomicOr(reinterpret_cast<unsigned long long *>(&orand[2 * D]), (unsigned long long)lo);
        atomicAnd(reinterpret_cast<unsigned long long *>(&orand[2 * D + 1]), (unsigned long long)la);
    }
    for (uint32_t d = 0; d < D; d++) {
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

// sort key of sorted position j for pass `d` (d == kNone: the key length)
__global__ __launch_bounds__(kMergeThreads) void merge_extract_kernel(MergeIn m, const uint32_t *perm,
                                                                      uint32_t d, uint64_t *keys) {
    const uint32_t j = blockIdx.x * kMergeThreads + threadIdx.x;
    if (j >= m.n) return;
    const uint32_t i = perm ? perm[j] : j;
    if (d == kNone) {
        keys[j] = key_len(m, i);
    } else {
        const View v = view(m, i);
        keys[j] = key_chunk(m.bytes + v.ko, v.kl, d);
    }
}

__global__ __launch_bounds__(kMergeThreads) void merge_iota_kernel(uint32_t *perm, uint32_t n) {
    const uint32_t j = blockIdx.x * kMergeThreads + threadIdx.x;
    if (j < n) perm[j] = j;
}

__device__ __forceinline__ bool keys_equal(const uint8_t *b, const View &x, const View &y) {
    if (x.kl != y.kl) return false;
    const uint8_t *p = b + x.ko, *q = b + y.ko;
    for (uint32_t t = 0; t < x.kl; t++)
        if (p[t] != q[t]) return false;
    return true;
}

__device__ __forceinline__ bool is_tombstone(const uint8_t *b, const View &v) {
    if (v.vl != 13) return false;
    const uint8_t *p = b + v.vo;
    for (int t = 0; t < 13; t++)
        if (p[t] != kTomb[t]) return false;
    return true;
}

// flags[j]: bit 0 = starts a group, bit 1 = may be written (not a tombstone
// dropped at level 6)
__global__ __launch_bounds__(kMergeThreads) void merge_flags_kernel(MergeIn m, const uint32_t *perm,
                                                                    int level, uint8_t *flags) {
    const uint32_t j = blockIdx.x * kMergeThreads + threadIdx.x;
    if (j >= m.n) return;
    const View v = view(m, perm[j]);
    bool gs = j == 0 || v.kl == 0;
    if (!gs) gs = !keys_equal(m.bytes, v, view(m, perm[j - 1]));
    const bool wr = level < 6 || !is_tombstone(m.bytes, v);
    flags[j] = (uint8_t)((gs ? 1 : 0) | (wr ? 2 : 0));
}

// candidate = the first pair of its group that may be written; the backward
// scan stops at the first writable pair or the group start, so each run of
// dropped tombstones is scanned by one pair only (O(n) in total)
__global__ __launch_bounds__(kMergeThreads) void merge_candidate_kernel(MergeIn m,
                                                                        const uint32_t *perm,
                                                                        const uint8_t *flags,
                                                                        uint32_t *csize,
                                                                        uint32_t *cflag) {
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
    uint32_t sz = 0;
    if (c) {
        const View v = view(m, perm[j]);
        sz = 16 + v.kl + v.vl;  // EstimateSize, kv.go:118-121
    }
    csize[j] = sz;
    cflag[j] = c ? 1u : 0u;
}

struct MergeFile {
    uint32_t p;      // first sorted position of the file
    uint32_t extra;  // sorted position of the group continuation written first, or kNone
    uint64_t o;      // first output slot
};

struct WalkArgs {
    MergeIn m;
    const uint32_t *perm;
    const uint8_t *flags;
    const uint64_t *S;  // exclusive scan of candidate sizes, n + 1
    const uint64_t *C;  // exclusive scan of candidate flags, n + 1
    uint64_t threshold;
    MergeFile *files;
    uint32_t *out;
    uint64_t *counts;   // [0] = written pairs, [1] = files
};

// smallest k in [lo, hi] with S[k] >= t, given S[hi] >= t; 64 probes a round
__device__ uint32_t wave_lower_bound(const uint64_t *S, uint32_t lo, uint32_t hi, uint64_t t,
                                     uint32_t guess) {
    const uint32_t lane = lane_id();
    if (guess >= lo && guess <= hi) {  // a window of 64 around the guess first
        uint32_t a = guess >= lo + 32 ? guess - 32 : lo;
        if (a + 63 > hi) a = hi >= lo + 63 ? hi - 63 : lo;
        const uint32_t k = a + lane <= hi ? a + lane : hi;
        const uint64_t ge = __ballot(S[k] >= t);
        if (ge & 1) {
            hi = a;
        } else if (ge) {
            return uni(a + (uint32_t)__builtin_ctzll(ge));
        } else {
            lo = a + 63 < hi ? a + 64 : hi;
        }
    }
    while (hi > lo) {
        // lane l probes lo + l*step, the last lane probes hi (S[hi] >= t), so
        // the first lane at or above t exists and the lane before it is below
        const uint32_t span = hi - lo;
        const uint32_t step = span >= 63 ? (span + 62) / 63 : 1;
        uint32_t k = lo + lane * step;
        if (k > hi || lane == kWave - 1) k = hi;
        const uint64_t ge = __ballot(S[k] >= t);
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
// size reaches the threshold.
__global__ __launch_bounds__(64) void merge_walk_kernel(WalkArgs a) {
    const uint32_t n = a.m.n, lane = lane_id();
    uint32_t p = 0, nf = 0, prev_span = 0;
    uint64_t o = 0;
    while (p < n) {
        uint32_t g = p, w = kNone;
        uint64_t wsize = 0;
        if (p > 0 && !(a.flags[p] & 1)) {
            // the rest of the group: its end and its first writable pair
            for (uint32_t q0 = p;; q0 += kWave) {
                const uint32_t q = q0 + lane;
                const uint8_t f = q < n ? a.flags[q] : 1;
                const bool end = q >= n || (q > p && (f & 1));
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
        }
        uint32_t e = kNone;  // sorted position of the pair that triggers the flush
        if (w != kNone && wsize >= a.threshold) {
            e = w;
        } else {
            const uint64_t t = a.S[g] + (a.threshold - wsize);
            if (a.S[n] >= t) {
                const uint32_t k = wave_lower_bound(a.S, g + 1, n, t, g + prev_span);
                e = k - 1;
            }
        }
        const uint32_t end = e == kNone ? n : e + 1;
        const uint64_t nw = (w != kNone ? 1 : 0) + (end > g ? a.C[end] - a.C[g] : 0);
        if (nw == 0) break;  // nothing left to write: no file (builder.size == 0)
        if (lane == 0) {
            a.files[nf] = MergeFile{p, w, o};
            if (w != kNone) a.out[o] = a.perm[w];
        }
        o += nw;
        nf++;
        prev_span = end - g;
        p = end;
    }
    if (lane == 0) {
        a.files[nf] = MergeFile{n, kNone, o};
        a.counts[0] = o;
        a.counts[1] = nf;
    }
}

// each candidate's output slot: its file's first slot, after the extra, plus
// the candidates before it in the file
__global__ __launch_bounds__(kMergeThreads) void merge_emit_kernel(
    const uint32_t *perm, const uint64_t *C, const uint32_t *cflag, const MergeFile *files,
    const uint64_t *counts, uint32_t n, uint32_t *out, uint64_t *file_start) {
    const uint32_t j = blockIdx.x * kMergeThreads + threadIdx.x;
    const uint32_t nf = (uint32_t)counts[1];
    if (j <= nf && file_start) file_start[j] = files[j].o;
    if (j >= n || !cflag[j]) return;
    uint32_t lo = 0, hi = nf;  // last file with p <= j
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (files[mid].p <= j) lo = mid; else hi = mid;
    }
    if (nf == 0 || files[lo].p > j || j >= files[lo + 1].p) return;  // past the last file
    const MergeFile F = files[lo];
    out[F.o + (F.extra != kNone ? 1 : 0) + (C[j] - C[F.p])] = perm[j];
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

// one wave per 64 pairs: the wave copies each pair's key and value in turn
__global__ __launch_bounds__(kMergeThreads) void gather_copy_kernel(
    MergeIn m, const uint32_t *idx, uint32_t nout, const uint64_t *koff, const uint64_t *voff,
    uint8_t *keys, uint8_t *vals) {
    const uint32_t j0 = (blockIdx.x * kMergeThreads + threadIdx.x) / kWave * kWave;
    if (j0 >= nout) return;
    const uint32_t lane = lane_id(), j = j0 + lane;
    View v{};
    uint64_t ko = 0, vo = 0;
    if (j < nout) {
        v = view(m, idx[j]);
        ko = koff[j];
        vo = voff[j];
    }
    const uint32_t cnt = nout - j0 < kWave ? nout - j0 : kWave;
    for (uint32_t r = 0; r < cnt; r++) {
        const uint64_t sk = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(v.ko >> 32), r) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((uint32_t)v.ko, r);
        const uint64_t sv = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(v.vo >> 32), r) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((uint32_t)v.vo, r);
        const uint32_t kl = __builtin_amdgcn_readlane(v.kl, r);
        const uint32_t vl = __builtin_amdgcn_readlane(v.vl, r);
        const uint64_t dk = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(ko >> 32), r) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((uint32_t)ko, r);
        const uint64_t dv = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(vo >> 32), r) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((uint32_t)vo, r);
        // resources start a dword before the bytes (keys and values sit at
        // rec_off + 4 or later) so wave_copy's offsets never wrap below 0
        const uint64_t ka = (sk & ~(uint64_t)3) - 4, va = (sv & ~(uint64_t)3) - 4;
        wave_copy(make_rsrc(m.bytes + ka, kl + 12), (uint32_t)(sk - ka), keys + dk, kl);
        wave_copy(make_rsrc(m.bytes + va, vl + 12), (uint32_t)(sv - va), vals + dv, vl);
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

struct MergeWs {
    uint32_t *perm[2];
    uint64_t *keys[2];
    uint8_t *flags;
    uint32_t *csize, *cflag;
    uint64_t *S, *C;
    MergeFile *files;
    uint64_t *stats;  // [0] max len, [1] min len, [2] counts (2 words), [4..] chunk OR/AND
    void *scan_ws;
    size_t scan_bytes;
    void *sort_tmp;
    size_t sort_bytes;
    size_t total;
};

size_t sort_tmp_bytes(uint32_t n) {
    size_t b = 0;
    (void)rocprim::radix_sort_pairs(nullptr, b, (uint64_t *)nullptr, (uint64_t *)nullptr,
                              (uint32_t *)nullptr, (uint32_t *)nullptr, n, 0, 64);
    return b;
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
    w.perm[0] = reinterpret_cast<uint32_t *>(take(4 * nn));
    w.perm[1] = reinterpret_cast<uint32_t *>(take(4 * nn));
    w.keys[0] = reinterpret_cast<uint64_t *>(take(8 * nn));
    w.keys[1] = reinterpret_cast<uint64_t *>(take(8 * nn));
    w.flags = take(nn);
    w.csize = reinterpret_cast<uint32_t *>(take(4 * nn));
    w.cflag = reinterpret_cast<uint32_t *>(take(4 * nn));
    w.S = reinterpret_cast<uint64_t *>(take(8 * (nn + 1)));
    w.C = reinterpret_cast<uint64_t *>(take(8 * (nn + 1)));
    w.files = reinterpret_cast<MergeFile *>(take(kFileBytes * (nn + 2)));
    w.stats = reinterpret_cast<uint64_t *>(take(8 * (4 + 2 * (size_t)kMaxChunks + 2)));
    w.scan_bytes = scan_workspace_bytes(n);
    w.scan_ws = take(w.scan_bytes);
    w.sort_bytes = sort_tmp_bytes(n);
    w.sort_tmp = take(w.sort_bytes);
    w.total = at;
    return w;
}

uint32_t grid_for(uint64_t n) { return (uint32_t)((n + kMergeThreads - 1) / kMergeThreads); }

}  // namespace
}  // namespace lsm

using namespace lsm;

static_assert(sizeof(MergeFile) == kFileBytes, "MergeFile layout");

extern "C" size_t lsm_merge_kvs_workspace_bytes(uint64_t n) {
    if (n >= 0xFFFFFFFFull) return 0;
    return merge_ws_layout(nullptr, (uint32_t)n).total;
}

extern "C" int lsm_merge_kvs(lsm_ctx *ctx, const uint8_t *d_bytes, const lsm_rec_desc *d_key_desc,
                             const lsm_rec_desc *d_val_desc, uint64_t n, int level,
                             uint64_t threshold, uint32_t *d_out, uint64_t *d_file_start,
                             uint64_t *h_counts, void *d_ws, size_t ws_bytes, void *stream) {
    if (!ctx || !h_counts || threshold == 0 || n >= 0xFFFFFFFFull) return LSM_EINVAL;
    if (n && (!d_bytes || !d_key_desc || !d_out || !d_ws)) return LSM_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    h_counts[0] = h_counts[1] = 0;
    if (n == 0) {
        if (d_file_start) LSM_HIP_CHECK(hipMemsetAsync(d_file_start, 0, 8, s));
        return 0;
    }
    const uint32_t N = (uint32_t)n;
    MergeWs w = merge_ws_layout(static_cast<uint8_t *>(d_ws), N);
    if (ws_bytes < w.total) return LSM_ESPACE;
    const MergeIn m{d_bytes, d_key_desc, d_val_desc, N};
    const uint32_t sb = grid_for(n) < kStatBlocks ? grid_for(n) : kStatBlocks;

    // 1. key lengths, then per-chunk statistics
    uint64_t init[2] = {0, ~0ull};
    LSM_HIP_CHECK(hipMemcpyAsync(w.stats, init, 16, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(merge_len_kernel, dim3(sb), dim3(kMergeThreads), 0, s, m, w.stats);
    uint64_t lens[2];
    LSM_HIP_CHECK(hipMemcpyAsync(lens, w.stats, 16, hipMemcpyDeviceToHost, s));
    LSM_HIP_CHECK(hipStreamSynchronize(s));
    const uint32_t D = (uint32_t)((lens[0] + 7) / 8), minlen = (uint32_t)lens[1];
    if (D > kMaxChunks) return LSM_EINVAL;
    uint64_t *orand = w.stats + 4;
    std::vector<uint64_t> st(2 * (size_t)D + 2);
    for (uint32_t d = 0; d <= D; d++) {
        st[2 * d] = 0;
        st[2 * d + 1] = ~0ull;
    }
    LSM_HIP_CHECK(hipMemcpyAsync(orand, st.data(), st.size() * 8, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(merge_chunk_stats_kernel, dim3(sb), dim3(kMergeThreads), 0, s, m, D, orand);
    LSM_HIP_CHECK(hipMemcpyAsync(st.data(), orand, st.size() * 8, hipMemcpyDeviceToHost, s));
    LSM_HIP_CHECK(hipStreamSynchronize(s));

    // 2. stable LSD passes: key length, then chunks D-1 .. 0 (varying bits only)
    int cur = 0;
    bool have_perm = false;
    auto pass = [&](uint32_t d, uint64_t vary) -> int {
        if (!vary) return 0;
        const int b0 = __builtin_ctzll(vary), b1 = 64 - __builtin_clzll(vary);
        hipLaunchKernelGGL(merge_extract_kernel, dim3(grid_for(n)), dim3(kMergeThreads), 0, s, m,
                           have_perm ? w.perm[cur] : nullptr, d, w.keys[0]);
        if (!have_perm) {
            hipLaunchKernelGGL(merge_iota_kernel, dim3(grid_for(n)), dim3(kMergeThreads), 0, s,
                               w.perm[cur], N);
            have_perm = true;
        }
        size_t tb = w.sort_bytes;
        const hipError_t e = rocprim::radix_sort_pairs(w.sort_tmp, tb, w.keys[0], w.keys[1],
                                                       w.perm[cur], w.perm[cur ^ 1], N, b0, b1, s);
        if (e != hipSuccess) return -(1000 + (int)e);
        cur ^= 1;
        return 0;
    };
    int rc = pass(kNone, st[2 * D] & ~st[2 * D + 1]);
    for (uint32_t d = D; rc == 0 && d-- > 0;) {
        const uint64_t and_d = minlen > 8 * d ? st[2 * d + 1] : 0;  // short keys hold 0
        rc = pass(d, st[2 * d] & ~and_d);
    }
    if (rc) return rc;
    if (!have_perm)
        hipLaunchKernelGGL(merge_iota_kernel, dim3(grid_for(n)), dim3(kMergeThreads), 0, s,
                           w.perm[cur], N);
    const uint32_t *perm = w.perm[cur];

    // 3. groups and candidates; 4. scans and the file walk; 5. emit
    hipLaunchKernelGGL(merge_flags_kernel, dim3(grid_for(n)), dim3(kMergeThreads), 0, s, m, perm,
                       level, w.flags);
    hipLaunchKernelGGL(merge_candidate_kernel, dim3(grid_for(n)), dim3(kMergeThreads), 0, s, m,
                       perm, w.flags, w.csize, w.cflag);
    rc = scan_u32_to_u64(w.csize, N, w.S, w.scan_ws, w.scan_bytes, s);
    if (!rc) rc = scan_u32_to_u64(w.cflag, N, w.C, w.scan_ws, w.scan_bytes, s);
    if (rc) return rc;
    WalkArgs wa{m, perm, w.flags, w.S, w.C, threshold, w.files, d_out, w.stats + 2};
    hipLaunchKernelGGL(merge_walk_kernel, dim3(1), dim3(64), 0, s, wa);
    hipLaunchKernelGGL(merge_emit_kernel, dim3(grid_for(n + 1)), dim3(kMergeThreads), 0, s, perm,
                       w.C, w.cflag, w.files, w.stats + 2, N, d_out, d_file_start);
    LSM_HIP_CHECK(hipGetLastError());
    LSM_HIP_CHECK(hipMemcpyAsync(h_counts, w.stats + 2, 16, hipMemcpyDeviceToHost, s));
    LSM_HIP_CHECK(hipStreamSynchronize(s));
    return 0;
}

extern "C" size_t lsm_gather_kvs_workspace_bytes(uint64_t nout) {
    const size_t nn = nout ? nout : 1;
    return 2 * ((4 * nn + 255) & ~(size_t)255) + scan_workspace_bytes((uint32_t)nout);
}

extern "C" int lsm_gather_kvs(lsm_ctx *ctx, const uint8_t *d_bytes, const lsm_rec_desc *d_key_desc,
                              const lsm_rec_desc *d_val_desc, const uint32_t *d_idx, uint64_t nout,
                              uint8_t *d_keys, uint64_t *d_koff, uint8_t *d_vals, uint64_t *d_voff,
                              void *d_ws, size_t ws_bytes, void *stream) {
    if (!ctx || !d_koff || !d_voff || nout >= 0xFFFFFFFFull) return LSM_EINVAL;
    if (nout && (!d_bytes || !d_key_desc || !d_idx || !d_keys || !d_vals || !d_ws))
        return LSM_EINVAL;
    if (ws_bytes < lsm_gather_kvs_workspace_bytes(nout)) return LSM_ESPACE;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint32_t N = (uint32_t)nout;
    const size_t nn = nout ? nout : 1, part = (4 * nn + 255) & ~(size_t)255;
    uint32_t *kl = static_cast<uint32_t *>(d_ws);
    uint32_t *vl = reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(d_ws) + part);
    void *sw = static_cast<uint8_t *>(d_ws) + 2 * part;
    const size_t sbytes = scan_workspace_bytes(N);
    const MergeIn m{d_bytes, d_key_desc, d_val_desc, N};
    if (N)
        hipLaunchKernelGGL(gather_lens_kernel, dim3(grid_for(nout)), dim3(kMergeThreads), 0, s, m,
                           d_idx, N, kl, vl);
    int rc = scan_u32_to_u64(kl, N, d_koff, sw, sbytes, s);
    if (!rc) rc = scan_u32_to_u64(vl, N, d_voff, sw, sbytes, s);
    if (rc) return rc;
    if (N)
        hipLaunchKernelGGL(gather_copy_kernel, dim3(grid_for(nout)), dim3(kMergeThreads), 0, s, m,
                           d_idx, N, d_koff, d_voff, d_keys, d_vals);
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
