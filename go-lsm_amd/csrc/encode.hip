// encode.hip — batched record encode, fused-bloom .sst build and bloom probe (gfx950).
//
// Encoding is output-centric.  With a CSR record batch every record's output
// position is closed-form (KV: 8*i + K(i) + V(i), V: 4*i + V(i), IDX:
// 12*i + K(i), relative to the region's first record), which is exactly
// SSTable.EncodeTo's exclusive prefix sum of 4+len (sstable.go:164-175)
// without a scan.  A wave takes a chunk of up to 64 records (one per lane,
// positions by a wave prefix sum), then every lane assembles whole aligned
// output dwords: the common dword lies inside one key/value and is two
// aligned source loads + v_alignbyte; dwords that straddle a length field
// are assembled byte by byte.  Chunk-edge dwords shared with a neighbour
// chunk are written with byte stores, everything else with dword stores.
//
// The bloom filter (1.6 Mbit in go-lsm) does not fit one CU's LDS, so each
// .sst's bitmap is built in LDS slices: one workgroup per (file, slice)
// hashes every key of the file (sum256 + 16 locations + Barrett modulo) and
// ds_or's the bits that fall in its slice; the slice is then stored once.
// No global atomics.
#include "common.h"
#include "murmur.h"

namespace lsm {
namespace {

struct RegionSrc {
    const uint8_t *keys;
    const uint64_t *koff;
    const uint8_t *vals;
    const uint64_t *voff;
    const int64_t *idx_off;  // IDX: per-record offsets (encode_blocks) or null
    int64_t idx_base;        // IDX (.sst): offset(i) = idx_base + 4*(i-rs) + V(i)-V(rs)
    uint64_t rs, vrs;
};

template <int G>
struct GrammarTraits;
template <>
struct GrammarTraits<LSM_GRAMMAR_V> { static constexpr uint32_t pre = 4; static constexpr bool K = false, V = true; };
template <>
struct GrammarTraits<LSM_GRAMMAR_KV> { static constexpr uint32_t pre = 8; static constexpr bool K = true, V = true; };
template <>
struct GrammarTraits<LSM_GRAMMAR_IDX> { static constexpr uint32_t pre = 12; static constexpr bool K = true, V = false; };

// Byte w of a record (w < record size).
template <int G>
__device__ __forceinline__ uint32_t rec_byte(const RegionSrc &S, uint64_t K0, uint32_t kl,
                                             uint64_t V0, uint32_t vl, int64_t xo, uint64_t w) {
    if (G == LSM_GRAMMAR_V) {
        if (w < 4) return (vl >> (8 * w)) & 0xff;
        return S.vals[V0 + w - 4];
    }
    if (w < 4) return (kl >> (8 * w)) & 0xff;
    if (w < 4 + (uint64_t)kl) return S.keys[K0 + w - 4];
    uint64_t w2 = w - 4 - kl;
    if (G == LSM_GRAMMAR_IDX) return (uint32_t)((uint64_t)xo >> (8 * w2)) & 0xff;
    if (w2 < 4) return (vl >> (8 * w2)) & 0xff;
    return S.vals[V0 + w2 - 4];
}

// Per-wave record table of one chunk (LDS).
struct ChunkTable {
    uint64_t P[kWave + 1];  // chunk-relative record starts; P[cnt] = chunk bytes
    uint64_t K0[kWave], V0[kWave];
    int64_t xo[kWave];
    uint32_t kl[kWave], vl[kWave];
};

// Encode records [c0, c0+cnt) (cnt <= 64) whose first byte goes to dst.
template <int G>
__device__ void encode_chunk(const RegionSrc &S, uint64_t c0, uint32_t cnt, uint8_t *dst,
                             ChunkTable *tb) {
    using T = GrammarTraits<G>;
    const uint32_t lane = lane_id();
    uint64_t K0 = 0, V0 = 0;
    uint32_t kl = 0, vl = 0;
    int64_t xo = 0;
    uint64_t sz = 0;
    if (lane < cnt) {
        uint64_t i = c0 + lane;
        if (T::K) { K0 = S.koff[i]; kl = (uint32_t)(S.koff[i + 1] - K0); }
        if (T::V || (G == LSM_GRAMMAR_IDX && !S.idx_off)) {
            V0 = S.voff[i];
            vl = (uint32_t)(S.voff[i + 1] - V0);
        }
        if (G == LSM_GRAMMAR_IDX)
            xo = S.idx_off ? S.idx_off[i]
                           : S.idx_base + (int64_t)(4 * (i - S.rs) + (V0 - S.vrs));
        sz = T::pre + (T::K ? kl : 0) + (T::V ? vl : 0);
    }
    uint64_t tot;
    const uint64_t P = wave_excl_scan64(sz, &tot);
    // Publish the table; a previous chunk's readers in this wave are done
    // (LDS ops of one wave execute in order).
    __builtin_amdgcn_wave_barrier();
    __asm__ __volatile__("" ::: "memory");
    if (lane < cnt) {
        tb->P[lane] = P;
        tb->K0[lane] = K0;
        tb->V0[lane] = V0;
        tb->xo[lane] = xo;
        tb->kl[lane] = kl;
        tb->vl[lane] = vl;
    }
    if (lane == 0) tb->P[cnt] = tot;
    __builtin_amdgcn_wave_barrier();
    __asm__ __volatile__("" ::: "memory");

    const uintptr_t Ob = reinterpret_cast<uintptr_t>(dst);
    const uint32_t head = (uint32_t)(Ob & 3);
    uint32_t *dA = reinterpret_cast<uint32_t *>(Ob - head);
    const uint64_t ndw = (head + tot + 3) >> 2;

    uint32_t r = 0;             // this lane's record cursor
    uint64_t Pn = tb->P[1 <= cnt ? 1 : 0];  // start of record r+1
    for (uint64_t d = lane; d < ndw; d += kWave) {
        const int64_t u0 = (int64_t)(4 * d) - head;
        const uint64_t uf = u0 < 0 ? 0 : (uint64_t)u0;
        while (r + 1 < cnt && Pn <= uf) {
            r++;
            Pn = tb->P[r + 1];
        }
        const bool full = u0 >= 0 && (uint64_t)u0 + 4 <= tot;
        const uint64_t Pr = tb->P[r];
        const uint32_t rkl = T::K ? tb->kl[r] : 0;
        uint32_t v = 0;
        bool fast = false;
        if (full) {
            const uint64_t w0 = (uint64_t)u0 - Pr;
            if (T::K && w0 >= 4 && w0 + 4 <= 4 + (uint64_t)rkl) {
                v = ldg_u32_unaligned(S.keys + tb->K0[r] + (w0 - 4));
                fast = true;
            } else if (G == LSM_GRAMMAR_KV && w0 >= 8 + (uint64_t)rkl &&
                       w0 + 4 <= 8 + (uint64_t)rkl + tb->vl[r]) {
                v = ldg_u32_unaligned(S.vals + tb->V0[r] + (w0 - 8 - rkl));
                fast = true;
            } else if (G == LSM_GRAMMAR_V && w0 >= 4 && w0 + 4 <= 4 + (uint64_t)tb->vl[r]) {
                v = ldg_u32_unaligned(S.vals + tb->V0[r] + (w0 - 4));
                fast = true;
            }
        }
        if (fast) {
            dA[d] = v;
            continue;
        }
        // Slow path (length fields, record boundaries, chunk edges): byte by byte.
        uint32_t rr = r;
        uint8_t *db = reinterpret_cast<uint8_t *>(dA + d);
        for (uint32_t t = 0; t < 4; t++) {
            const int64_t u = u0 + t;
            if (u < 0 || (uint64_t)u >= tot) continue;
            while (rr + 1 < cnt && tb->P[rr + 1] <= (uint64_t)u) rr++;
            const uint32_t byte = rec_byte<G>(S, tb->K0[rr], tb->kl[rr], tb->V0[rr], tb->vl[rr],
                                              tb->xo[rr], (uint64_t)u - tb->P[rr]);
            if (full) v |= byte << (8 * t);
            else db[t] = (uint8_t)byte;
        }
        if (full) dA[d] = v;
    }
}

// ---- lsm_encode_blocks ----------------------------------------------------

struct EncodeBlocksArgs {
    RegionSrc S;
    const uint64_t *rec_start;
    uint32_t nblk;
    uint8_t *out;
    const uint64_t *out_off;
};

constexpr int kEncWaves = 4;

template <int G>
__global__ __launch_bounds__(256) void encode_blocks_kernel(EncodeBlocksArgs a) {
    using T = GrammarTraits<G>;
    __shared__ ChunkTable tables[kEncWaves];
    const uint32_t b = blockIdx.x;
    const uint32_t wave = uni(threadIdx.x / kWave);
    const uint64_t rs = uni64(a.rec_start[b]);
    const uint64_t re = uni64(a.rec_start[b + 1]);
    uint8_t *out = a.out + uni64(a.out_off[b]);
    const uint64_t Krs = T::K ? uni64(a.S.koff[rs]) : 0;
    const uint64_t Vrs = T::V ? uni64(a.S.voff[rs]) : 0;
    for (uint64_t c0 = rs + (uint64_t)wave * kWave; c0 < re; c0 += kEncWaves * kWave) {
        uint32_t cnt = (uint32_t)((re - c0) < (uint64_t)kWave ? (re - c0) : kWave);
        uint64_t rel = T::pre * (c0 - rs);
        if (T::K) rel += uni64(a.S.koff[c0]) - Krs;
        if (T::V) rel += uni64(a.S.voff[c0]) - Vrs;
        encode_chunk<G>(a.S, c0, cnt, out + rel, &tables[wave]);
    }
}

// ---- fused bloom build (LDS slices) --------------------------------------

struct BloomArgs {
    const uint8_t *keys;
    const uint64_t *koff;
    const uint64_t *file_start;
    uint64_t m, mrecip;
    uint32_t k;
    uint64_t slice_bits;   // multiple of 64
    uint64_t nwords;       // ceil(m/64)
    uint64_t *bitmap;      // nfile * nwords native u64 words
    uint64_t nkeys;        // keys of the single filter when file_start == null
};

__global__ __launch_bounds__(1024) void bloom_slices_kernel(BloomArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_bits[];
    const uint32_t f = blockIdx.x;
    const uint64_t lo = (uint64_t)blockIdx.y * a.slice_bits;
    if (lo >= a.m) return;
    const uint64_t hi = lo + a.slice_bits < a.m ? lo + a.slice_bits : a.m;
    const uint32_t nw32 = (uint32_t)((hi - lo + 63) / 64) * 2;
    for (uint32_t i = threadIdx.x; i < nw32; i += blockDim.x) lds_bits[i] = 0;
    __syncthreads();
    const uint64_t s = a.file_start ? a.file_start[f] : 0;
    const uint64_t e = a.file_start ? a.file_start[f + 1] : a.nkeys;
    for (uint64_t i = s + threadIdx.x; i < e; i += blockDim.x) {
        uint64_t k0 = a.koff[i];
        uint64_t h[4];
        sum256(a.keys + k0, a.koff[i + 1] - k0, h);
        for (uint32_t j = 0; j < a.k; j++) {
            uint64_t p = mod_barrett(location(h, j), a.m, a.mrecip);
            if (p >= lo && p < hi) {
                uint32_t q = (uint32_t)(p - lo);
                atomicOr(&lds_bits[q >> 5], 1u << (q & 31));
            }
        }
    }
    __syncthreads();
    uint32_t *dst = reinterpret_cast<uint32_t *>(a.bitmap + (uint64_t)f * a.nwords + lo / 64);
    for (uint32_t i = threadIdx.x; i < nw32; i += blockDim.x) dst[i] = lds_bits[i];
}

// ---- .sst image writer ------------------------------------------------------

struct SstArgs {
    const uint8_t *keys;
    const uint64_t *koff;
    const uint8_t *vals;
    const uint64_t *voff;
    const uint64_t *file_start;
    uint8_t *out;
    const uint64_t *file_off;
    int64_t *footer;
    const uint64_t *bitmap;
    uint64_t m, nwords;
    uint32_t k;
};

struct SstLayout {
    uint64_t s, e;
    uint32_t kl0, kl1;
    uint64_t hdr, filter_bytes, data_off, data_size, idx_off, idx_size, img;
};

__device__ __forceinline__ SstLayout sst_layout(const SstArgs &a, uint32_t f) {
    SstLayout L;
    L.s = uni64(a.file_start[f]);
    L.e = uni64(a.file_start[f + 1]);
    L.kl0 = L.kl1 = 0;
    if (L.e > L.s) {
        L.kl0 = (uint32_t)(uni64(a.koff[L.s + 1]) - uni64(a.koff[L.s]));
        L.kl1 = (uint32_t)(uni64(a.koff[L.e]) - uni64(a.koff[L.e - 1]));
    }
    L.hdr = 8 + (uint64_t)L.kl0 + L.kl1;
    L.filter_bytes = 32 + 8 * a.nwords;
    L.data_off = L.hdr + L.filter_bytes;
    const uint64_t n = L.e - L.s;
    L.data_size = 4 * n + (uni64(a.voff[L.e]) - uni64(a.voff[L.s]));
    L.idx_off = L.data_off + L.data_size;
    L.idx_size = 12 * n + (uni64(a.koff[L.e]) - uni64(a.koff[L.s]));
    L.img = L.idx_off + L.idx_size + 32;
    return L;
}

constexpr int kSstWaves = 4;
constexpr uint32_t kSstChunkRecs = kSstWaves * kWave;  // records per workgroup

// Data region (V grammar) and index region (IDX grammar) of file blockIdx.x,
// records chunk blockIdx.y.
__global__ __launch_bounds__(256) void sst_regions_kernel(SstArgs a) {
    __shared__ ChunkTable tables[kSstWaves];
    const uint32_t f = blockIdx.x;
    const SstLayout L = sst_layout(a, f);
    const uint32_t wave = uni(threadIdx.x / kWave);
    const uint64_t c0 = L.s + (uint64_t)blockIdx.y * kSstChunkRecs + (uint64_t)wave * kWave;
    if (c0 >= L.e) return;
    const uint32_t cnt = (uint32_t)((L.e - c0) < (uint64_t)kWave ? (L.e - c0) : kWave);
    uint8_t *img = a.out + uni64(a.file_off[f]);
    const uint64_t Ks = uni64(a.koff[L.s]), Vs = uni64(a.voff[L.s]);
    const uint64_t Kc = uni64(a.koff[c0]), Vc = uni64(a.voff[c0]);
    RegionSrc S;
    S.keys = a.keys; S.koff = a.koff; S.vals = a.vals; S.voff = a.voff;
    S.idx_off = nullptr;
    S.idx_base = (int64_t)L.data_off;
    S.rs = L.s;
    S.vrs = Vs;
    encode_chunk<LSM_GRAMMAR_V>(S, c0, cnt, img + L.data_off + 4 * (c0 - L.s) + (Vc - Vs),
                                 &tables[wave]);
    encode_chunk<LSM_GRAMMAR_IDX>(S, c0, cnt, img + L.idx_off + 12 * (c0 - L.s) + (Kc - Ks),
                                   &tables[wave]);
}

// Header | filter block | footer of file blockIdx.x.  The header+filter
// prefix [0, data_off) is cut into 4 KiB tiles over blockIdx.y; tile 0 also
// writes the footer.
constexpr uint32_t kMetaTile = 4096;

__device__ __forceinline__ uint32_t meta_byte(const SstArgs &a, const SstLayout &L,
                                              uint64_t fwords, uint64_t q) {
    // Header: u32 kl0 | key[s] | u32 kl1 | key[e-1]   (header.go:25-37)
    if (q < 4) return (L.kl0 >> (8 * q)) & 0xff;
    if (q < 4 + (uint64_t)L.kl0) return a.keys[a.koff[L.s] + q - 4];
    if (q < 8 + (uint64_t)L.kl0) return (L.kl1 >> (8 * (q - 4 - L.kl0))) & 0xff;
    if (q < L.hdr) return a.keys[a.koff[L.e - 1] + q - 8 - L.kl0];
    // Filter block (bloom.go:472-491): u64le L | u64be m | u64be k | u64be nbits | words be
    uint64_t r = q - L.hdr;
    uint64_t v;
    uint32_t be;
    if (r < 8) { v = 24 + 8 * a.nwords; return (uint32_t)(v >> (8 * r)) & 0xff; }
    r -= 8;
    uint64_t fi = r / 8, fb = r % 8;
    if (fi == 0) v = a.m;
    else if (fi == 1) v = a.k ? a.k : 1;
    else if (fi == 2) v = a.m;
    else v = a.bitmap[fwords + fi - 3];
    be = (uint32_t)(v >> (8 * (7 - fb))) & 0xff;
    return be;
}

__global__ __launch_bounds__(256) void sst_meta_kernel(SstArgs a) {
    const uint32_t f = blockIdx.x;
    const SstLayout L = sst_layout(a, f);
    uint8_t *img = a.out + uni64(a.file_off[f]);
    const uint64_t fwords = (uint64_t)f * a.nwords;
    const uint64_t t0 = (uint64_t)blockIdx.y * kMetaTile;
    if (t0 < L.data_off) {
        const uint64_t t1 = t0 + kMetaTile < L.data_off ? t0 + kMetaTile : L.data_off;
        const uintptr_t base = reinterpret_cast<uintptr_t>(img) + t0;
        const uint32_t head = (uint32_t)(base & 3);
        uint32_t *dA = reinterpret_cast<uint32_t *>(base - head);
        const uint64_t len = t1 - t0;
        const uint64_t ndw = (head + len + 3) / 4;
        for (uint64_t d = threadIdx.x; d < ndw; d += blockDim.x) {
            const int64_t u0 = (int64_t)(4 * d) - head;
            const bool full = u0 >= 0 && (uint64_t)u0 + 4 <= len;
            uint32_t v = 0;
            uint8_t *db = reinterpret_cast<uint8_t *>(dA + d);
            for (uint32_t t = 0; t < 4; t++) {
                int64_t u = u0 + t;
                if (u < 0 || (uint64_t)u >= len) continue;
                uint32_t byte = meta_byte(a, L, fwords, t0 + (uint64_t)u);
                if (full) v |= byte << (8 * t);
                else db[t] = (uint8_t)byte;
            }
            if (full) dA[d] = v;
        }
    }
    if (blockIdx.y == 0 && threadIdx.x < 32) {
        // Footer (footer.go:43-55): dataOff, dataSize, idxOff, idxSize (i64le)
        const uint32_t t = threadIdx.x;
        const uint64_t vals[4] = {L.data_off, L.data_size, L.idx_off, L.idx_size};
        img[L.img - 32 + t] = (uint8_t)(vals[t / 8] >> (8 * (t % 8)));
        if (a.footer && t < 4) a.footer[4 * (uint64_t)f + t] = (int64_t)vals[t];
    }
}

// ---- probe / hash ----------------------------------------------------------

__global__ __launch_bounds__(256) void sum256_kernel(const uint8_t *keys, const uint64_t *koff,
                                                     uint64_t n, uint64_t *out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t h[4];
    uint64_t k0 = koff[i];
    sum256(keys + k0, koff[i + 1] - k0, h);
    for (int j = 0; j < 4; j++) out[4 * i + j] = h[j];
}

__global__ __launch_bounds__(256) void bloom_probe_kernel(const uint64_t *words, uint64_t m,
                                                          uint64_t mrecip, uint32_t k,
                                                          const uint8_t *keys,
                                                          const uint64_t *koff, uint64_t n,
                                                          uint8_t *hit) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t h[4];
    uint64_t k0 = koff[i];
    sum256(keys + k0, koff[i + 1] - k0, h);
    uint8_t ok = 1;
    for (uint32_t j = 0; j < k && ok; j++) {
        uint64_t p = mod_barrett(location(h, j), m, mrecip);
        if (!((words[p >> 6] >> (p & 63)) & 1)) ok = 0;
    }
    hit[i] = ok;
}

template <int G>
int launch_encode_blocks(const EncodeBlocksArgs &a, hipStream_t s) {
    hipLaunchKernelGGL(encode_blocks_kernel<G>, dim3(a.nblk), dim3(kWave * kEncWaves), 0, s, a);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}

constexpr uint64_t kSliceBitsMax = 100ull * 1024 * 8;  // 100 KiB of LDS per slice

uint64_t slice_bits_for(uint64_t m) {
    uint64_t nslices = (m + kSliceBitsMax - 1) / kSliceBitsMax;
    if (nslices == 0) nslices = 1;
    uint64_t sb = (m + nslices - 1) / nslices;
    return (sb + 63) / 64 * 64;
}

}  // namespace
}  // namespace lsm

using namespace lsm;

extern "C" uint64_t lsm_encoded_size_host(int grammar, const uint64_t *koff, const uint64_t *voff,
                                          uint64_t r0, uint64_t r1) {
    uint64_t n = r1 - r0;
    switch (grammar) {
    case LSM_GRAMMAR_V: return 4 * n + (voff[r1] - voff[r0]);
    case LSM_GRAMMAR_KV: return 8 * n + (koff[r1] - koff[r0]) + (voff[r1] - voff[r0]);
    case LSM_GRAMMAR_IDX: return 12 * n + (koff[r1] - koff[r0]);
    default: return 0;
    }
}

extern "C" int lsm_encode_blocks(lsm_ctx *ctx, int grammar, const uint8_t *d_keys,
                                 const uint64_t *d_koff, const uint8_t *d_vals,
                                 const uint64_t *d_voff, const int64_t *d_idx_off,
                                 const uint64_t *d_rec_start, uint32_t nblk, uint8_t *d_out,
                                 const uint64_t *d_out_off, void *stream) {
    if (!ctx) return LSM_EINVAL;
    if (nblk == 0) return 0;
    if (!d_rec_start || !d_out || !d_out_off) return LSM_EINVAL;
    if (grammar < LSM_GRAMMAR_V || grammar > LSM_GRAMMAR_IDX) return LSM_EINVAL;
    if (grammar != LSM_GRAMMAR_V && (!d_keys || !d_koff)) return LSM_EINVAL;
    if (grammar != LSM_GRAMMAR_IDX && (!d_vals || !d_voff)) return LSM_EINVAL;
    if (grammar == LSM_GRAMMAR_IDX && !d_idx_off) return LSM_EINVAL;
    EncodeBlocksArgs a;
    a.S.keys = d_keys;
    a.S.koff = d_koff;
    a.S.vals = d_vals;
    a.S.voff = d_voff;
    a.S.idx_off = d_idx_off;
    a.S.idx_base = 0;
    a.S.rs = 0;
    a.S.vrs = 0;
    a.rec_start = d_rec_start;
    a.nblk = nblk;
    a.out = d_out;
    a.out_off = d_out_off;
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (grammar) {
    case LSM_GRAMMAR_V: return launch_encode_blocks<LSM_GRAMMAR_V>(a, s);
    case LSM_GRAMMAR_KV: return launch_encode_blocks<LSM_GRAMMAR_KV>(a, s);
    default: return launch_encode_blocks<LSM_GRAMMAR_IDX>(a, s);
    }
}

extern "C" uint64_t lsm_filter_block_size(uint64_t m) { return 32 + 8 * ((m + 63) / 64); }

extern "C" uint64_t lsm_segment_files_host(const uint64_t *koff, const uint64_t *voff, uint64_t n,
                                           uint64_t threshold, uint64_t *file_start) {
    // Builder.Add accumulates EstimateSize = 4+k+4+v+8 (kv.go:118-121) and the
    // driver flushes once size >= threshold (builder.go:40-42, merge.go:118-121);
    // leftovers form a last file (merge.go:125-128).  The running size of a file
    // starting at record s after record j is 16*(j+1-s) + K(j+1)-K(s) +
    // V(j+1)-V(s), monotone in j, so each boundary is a binary search.
    uint64_t nf = 0, s = 0;
    while (s < n) {
        file_start[nf++] = s;
        if (!threshold) { s = n; break; }
        const uint64_t base = 16 * s + koff[s] + voff[s];
        // smallest t in (s, n] with 16t + K(t) + V(t) - base >= threshold
        uint64_t lo = s + 1, hi = n + 1;
        while (lo < hi) {
            uint64_t mid = lo + (hi - lo) / 2;
            if (16 * mid + koff[mid] + voff[mid] - base >= threshold) hi = mid;
            else lo = mid + 1;
        }
        s = lo > n ? n : lo;
    }
    file_start[nf] = n;
    return nf;
}

extern "C" uint64_t lsm_sst_image_size_host(const uint64_t *koff, const uint64_t *voff,
                                            uint64_t r0, uint64_t r1, uint64_t m) {
    uint64_t hdr = 8;
    if (r1 > r0) hdr += (koff[r0 + 1] - koff[r0]) + (koff[r1] - koff[r1 - 1]);
    return hdr + lsm_filter_block_size(m) + lsm_encoded_size_host(LSM_GRAMMAR_V, koff, voff, r0, r1) +
           lsm_encoded_size_host(LSM_GRAMMAR_IDX, koff, voff, r0, r1) + 32;
}

extern "C" size_t lsm_build_sst_workspace_bytes(uint32_t nfile, uint64_t m) {
    uint64_t nw = (m + 63) / 64;
    return (size_t)(nfile ? nfile : 1) * (nw ? nw : 1) * 8;
}

static uint64_t barrett_recip(uint64_t m) { return ~0ull / m; }

extern "C" int lsm_build_sst(lsm_ctx *ctx, const uint8_t *d_keys, const uint64_t *d_koff,
                             const uint8_t *d_vals, const uint64_t *d_voff,
                             const uint64_t *d_file_start, uint32_t nfile,
                             uint32_t max_file_records, uint64_t m, uint32_t k, uint8_t *d_out,
                             const uint64_t *d_file_off, int64_t *d_footer, void *d_workspace,
                             size_t ws_bytes, void *stream) {
    if (!ctx || m == 0 || m >= (1ull << 63)) return LSM_EINVAL;
    if (nfile == 0) return 0;
    if (!d_keys || !d_koff || !d_vals || !d_voff || !d_file_start || !d_out || !d_file_off)
        return LSM_EINVAL;
    if (ws_bytes < lsm_build_sst_workspace_bytes(nfile, m) || !d_workspace) return LSM_ESPACE;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint64_t nwords = (m + 63) / 64;
    const uint32_t kk = k ? k : 1;  // NewBloomFilter max(1, k) bloom.go:95-101

    BloomArgs b;
    b.keys = d_keys;
    b.koff = d_koff;
    b.file_start = d_file_start;
    b.m = m;
    b.mrecip = barrett_recip(m);
    b.k = kk;
    b.slice_bits = slice_bits_for(m);
    b.nwords = nwords;
    b.bitmap = static_cast<uint64_t *>(d_workspace);
    b.nkeys = 0;
    const uint32_t nslices = (uint32_t)((m + b.slice_bits - 1) / b.slice_bits);
    const size_t lds = (size_t)(b.slice_bits / 8);
    hipLaunchKernelGGL(bloom_slices_kernel, dim3(nfile, nslices), dim3(1024), lds, s, b);
    LSM_HIP_CHECK(hipGetLastError());

    SstArgs a;
    a.keys = d_keys;
    a.koff = d_koff;
    a.vals = d_vals;
    a.voff = d_voff;
    a.file_start = d_file_start;
    a.out = d_out;
    a.file_off = d_file_off;
    a.footer = d_footer;
    a.bitmap = b.bitmap;
    a.m = m;
    a.nwords = nwords;
    a.k = kk;
    const uint32_t chunks = (max_file_records + kSstChunkRecs - 1) / kSstChunkRecs;
    if (chunks) {
        hipLaunchKernelGGL(sst_regions_kernel, dim3(nfile, chunks), dim3(256), 0, s, a);
        LSM_HIP_CHECK(hipGetLastError());
    }
    // header + filter tiles: the key lengths of the header are data-dependent;
    // bound the prefix by the max header (2 keys <= 2 * 2^20 + 8 is the
    // decode cap, but in practice keys are short) -- use the filter size plus
    // a generous header allowance and let tiles past data_off exit.
    const uint64_t prefix_max = lsm_filter_block_size(m) + 8 + 2 * 65536;
    const uint32_t tiles = (uint32_t)((prefix_max + kMetaTile - 1) / kMetaTile);
    hipLaunchKernelGGL(sst_meta_kernel, dim3(nfile, tiles), dim3(256), 0, s, a);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}

extern "C" int lsm_bloom_probe(lsm_ctx *ctx, const uint64_t *d_words, uint64_t m, uint32_t k,
                               const uint8_t *d_keys, const uint64_t *d_koff, uint64_t nkeys,
                               uint8_t *d_hit, void *stream) {
    if (!ctx || m == 0 || m >= (1ull << 63)) return LSM_EINVAL;
    if (nkeys == 0) return 0;
    if (!d_words || !d_keys || !d_koff || !d_hit) return LSM_EINVAL;
    uint32_t grid = (uint32_t)((nkeys + 255) / 256);
    hipLaunchKernelGGL(bloom_probe_kernel, dim3(grid), dim3(256), 0,
                       static_cast<hipStream_t>(stream), d_words, m, barrett_recip(m), k ? k : 1,
                       d_keys, d_koff, nkeys, d_hit);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}

extern "C" int lsm_sum256(lsm_ctx *ctx, const uint8_t *d_keys, const uint64_t *d_koff,
                          uint64_t nkeys, uint64_t *d_h, void *stream) {
    if (!ctx) return LSM_EINVAL;
    if (nkeys == 0) return 0;
    if (!d_keys || !d_koff || !d_h) return LSM_EINVAL;
    uint32_t grid = (uint32_t)((nkeys + 255) / 256);
    hipLaunchKernelGGL(sum256_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                       d_keys, d_koff, nkeys, d_h);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}

extern "C" int lsm_bloom_build(lsm_ctx *ctx, const uint8_t *d_keys, const uint64_t *d_koff,
                               uint64_t nkeys, uint64_t m, uint32_t k, uint64_t *d_words,
                               void *stream) {
    if (!ctx || m == 0 || m >= (1ull << 63) || !d_words) return LSM_EINVAL;
    if (nkeys && (!d_keys || !d_koff)) return LSM_EINVAL;
    BloomArgs b;
    b.keys = d_keys;
    b.koff = d_koff;
    b.file_start = nullptr;
    b.m = m;
    b.mrecip = barrett_recip(m);
    b.k = k ? k : 1;
    b.slice_bits = slice_bits_for(m);
    b.nwords = (m + 63) / 64;
    b.bitmap = d_words;
    b.nkeys = nkeys;
    const uint32_t nslices = (uint32_t)((m + b.slice_bits - 1) / b.slice_bits);
    hipLaunchKernelGGL(bloom_slices_kernel, dim3(1, nslices), dim3(1024),
                       (size_t)(b.slice_bits / 8), static_cast<hipStream_t>(stream), b);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}
