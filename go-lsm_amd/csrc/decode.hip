// decode.hip — batched record decode of length-prefixed blocks on gfx950.
//
// One wavefront owns one block (go-lsm's blocks are independent units; the
// parallelism is across blocks).  The block is streamed into a
// 4 KiB per-wave LDS ring in 1 KiB chunks (one coalesced 16 B/lane LDS-DMA
// buffer load each, range-checked so a block never reads past its padded end).  The
// record boundaries are a dependent chain (each record's position depends on
// every earlier length, data.go:58-76), so the wave chases them with a
// wave-uniform cursor: a window read (one ds_read_b128 per lane) exposes 1 KiB
// of the block across the wave's registers, and every length field inside it
// is two v_readlane plus a scalar funnel shift, i.e. one LDS round trip per
// 1 KiB instead of one per field.  Thirty-two waves per CU chase
// concurrently, which hides the LDS latency of the chain behind the HBM
// stream.  Decoded records are staged one per lane and written as coalesced
// 16-byte descriptors every 64 records.
#include <stdlib.h>
#include <string.h>

#include "common.h"

namespace lsm {
namespace {

constexpr int kWavesPerWG = 4;
constexpr uint32_t kRingBytes = 4096;
constexpr uint32_t kRingWords = kRingBytes / 4;
constexpr uint32_t kChunk = 1024;  // one b128 wave-load
constexpr uint32_t kNChunk = kRingBytes / kChunk;
constexpr uint32_t kSlotBytes = 4096;              // whole-block LDS slot
constexpr uint32_t kSlotStride = kSlotBytes + 16;  // skewed: lanes hit different banks
// Cache policy of the block loads: nt (streaming).  Each block byte is read
// once; keeping the stream out of the L2/MALL's normal replacement measured
// 80.5 -> 71.7 us for decode4k's memory pattern (tools/block_probe.py).
constexpr int kBlockLoadAux = 2;

#ifdef LSM_STAMPS
// Diagnostic build only (liblsm_gpu_stamps.so): per-workgroup s_memrealtime
// stamps {start, DMA landed, chase done, end} into a buffer of their own.
__device__ uint64_t *g_stamps;
__device__ __forceinline__ void stamp(uint32_t k) {
    if (threadIdx.x == 0 && g_stamps) g_stamps[blockIdx.x * 4 + k] = __builtin_amdgcn_s_memrealtime();
}
#else
__device__ __forceinline__ void stamp(uint32_t) {}
#endif

struct DecodeArgs {
    const uint8_t *in;
    const uint64_t *blk_off;
    const uint32_t *blk_len;
    uint32_t nblk;
    u32x4 *desc;
    const uint64_t *rec_base;
    uint32_t *nrec;
    int32_t *status;
    int64_t *idx_value;
    uint8_t *key_arena;
    uint8_t *val_arena;
    const uint64_t *arena_base;
    uint64_t *key_arena_off;
    uint64_t *val_arena_off;
};

// Streams one block through this wave's LDS ring and serves u32 length
// fields at wave-uniform block positions.
//
// Ring: 4 x 1 KiB chunks, filled by LDS-DMA (buffer_load_dwordx4 ... lds:
// no VGPR staging, one s_waitcnt for all chunks of a refill).  Window: each
// lane holds 16 raw bytes of a 1 KiB, 16-byte aligned slice of the stream
// (one ds_read_b128); a field at stream byte s is two v_readlane of the
// lanes/dwords covering [s, s+4) plus a scalar funnel shift.  A 4 KiB block
// costs ~5 LDS round trips instead of one per record.
struct BlockReader {
    uint32_t *ring;
    rsrc_t rsrc;
    uint32_t h;        // block start inside its first 16-byte line
    uint32_t total;    // loadable stream bytes: round_up16(h + n)
    uint32_t nchunks;  // chunks covering [0, total)
    uint32_t hi_c;     // chunks [.., hi_c) have been loaded into the ring
    uint32_t wb;       // window base (stream byte, 16-aligned)
    u32x4 raw;         // lane j: stream bytes [wb + 16j, wb + 16j + 16)
    bool have_win;

    __device__ void init(uint32_t *ring_, const uint8_t *in, uint64_t off, uint32_t n) {
        ring = ring_;
        uint64_t a0 = off & ~(uint64_t)15;
        h = (uint32_t)(off - a0);
        uint64_t tot = ((uint64_t)h + n + 15) & ~(uint64_t)15;
        total = (uint32_t)(tot > 0xFFFFFFF0ull ? 0xFFFFFFF0ull : tot);
        nchunks = (total + kChunk - 1) / kChunk;
        rsrc = make_rsrc(in + a0, total);
        hi_c = 0;
        have_win = false;
        wb = 0;
    }

    // Make stream bytes [s0, s0 + kChunk) resident (clamped to the block),
    // loading every missing chunk up to 3 chunks past s0's chunk.
    __device__ __forceinline__ void ensure(uint32_t s0) {
        uint32_t need_end = s0 + kChunk;
        if (need_end > total) need_end = total;
        const uint32_t need_hi = (need_end + kChunk - 1) / kChunk;
        if (need_hi <= hi_c) return;
        const uint32_t c0 = s0 / kChunk;
        const uint32_t first = hi_c > c0 ? hi_c : c0;
        uint32_t last = c0 + kNChunk;
        if (last > nchunks) last = nchunks;
        const uint32_t voff = lane_id() * 16;
#pragma unroll
        for (uint32_t i = 0; i < kNChunk; i++) {
            const uint32_t c = first + i;
            if (c < last)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rsrc, (__attribute__((address_space(3))) void *)&ring[(c % kNChunk) * (kChunk / 4)],
                    16, voff + c * kChunk, 0, 0, kBlockLoadAux);
        }
        hi_c = last;
        // The DMA writes are invisible to the compiler's waitcnt tracking of
        // ds_read; wait for them explicitly before the window read.
        __asm__ __volatile__("s_waitcnt vmcnt(0)" ::: "memory");
    }

    __device__ __forceinline__ void load_window(uint32_t s) {
        wb = s & ~15u;
        ensure(wb);
        const uint32_t w = ((wb + lane_id() * 16) % kRingBytes) / 4;
        raw = *reinterpret_cast<const u32x4 *>(&ring[w]);
        have_win = true;
    }

    // Dword d of lane l of the window (d, l wave-uniform).
    __device__ __forceinline__ uint32_t pick(uint32_t d, uint32_t l) const {
        uint32_t v0 = __builtin_amdgcn_readlane(raw.x, l);
        uint32_t v1 = __builtin_amdgcn_readlane(raw.y, l);
        uint32_t v2 = __builtin_amdgcn_readlane(raw.z, l);
        uint32_t v3 = __builtin_amdgcn_readlane(raw.w, l);
        return d == 0 ? v0 : d == 1 ? v1 : d == 2 ? v2 : v3;
    }

    // Little-endian u32 at block position p (wave-uniform).
    __device__ __forceinline__ uint32_t field(uint32_t p) {
        const uint32_t s = h + p;
        if (!have_win || s - wb > kChunk - 4) load_window(s);
        const uint32_t o = s - wb;
        const uint32_t l = o >> 4, d = (o >> 2) & 3, sh = o & 3;
        uint32_t lo = pick(d, l);
        if (sh) {
            const uint32_t hi = pick((d + 1) & 3, l + (d == 3));
            lo = (lo >> (8 * sh)) | (hi << (32 - 8 * sh));
        }
        return lo;
    }
};

// Records staged one per lane until 64 are ready, then stored coalesced.
struct RecordStage {
    uint32_t off_lo, off_hi, klen, vlen, x_lo, x_hi;

    __device__ __forceinline__ void put(uint32_t slot, uint64_t off, uint32_t k, uint32_t v,
                                        uint64_t x) {
        if (lane_id() == slot) {
            off_lo = (uint32_t)off;
            off_hi = (uint32_t)(off >> 32);
            klen = k;
            vlen = v;
            x_lo = (uint32_t)x;
            x_hi = (uint32_t)(x >> 32);
        }
    }
};

template <int G>
__device__ __forceinline__ void flush(const DecodeArgs &a, const RecordStage &st, uint64_t base,
                                      uint32_t first, uint32_t cnt) {
    uint32_t lane = lane_id();
    if (lane < cnt) {
        uint64_t i = base + first + lane;
        u32x4 d;
        d.x = st.off_lo;
        d.y = st.off_hi;
        d.z = st.klen;
        d.w = st.vlen;
        a.desc[i] = d;
        if (G == LSM_GRAMMAR_IDX && a.idx_value)
            a.idx_value[i] = (int64_t)((uint64_t)st.x_hi << 32 | st.x_lo);
    }
}

template <int G>
struct MinRecord { static constexpr uint32_t R = G == LSM_GRAMMAR_V ? 4 : G == LSM_GRAMMAR_KV ? 8 : 12; };

// Record slots: CSR rec_base, or offset-addressed (rec_base == NULL): block b
// owns slots [off/R, (off+n)/R) with R the grammar's minimum record size,
// disjoint for non-overlapping blocks -- no scan needed.
template <int G>
__device__ __forceinline__ void record_slots(const DecodeArgs &a, uint32_t b, uint64_t off,
                                             uint32_t n, uint64_t &base, uint64_t &cap) {
    constexpr uint32_t R = MinRecord<G>::R;
    if (a.rec_base) {
        base = a.rec_base[b];
        cap = a.rec_base[b + 1] - base;
    } else {
        base = off / R;
        cap = (off + n) / R - base;
    }
}

// Wave-per-block path: the whole wave chases one block (any size) through a
// 4 KiB LDS ring with a wave-uniform (scalar) cursor.  Used for ARENA mode and
// for blocks too large for a lane slot.
template <int G, bool ARENA>
__device__ void decode_block_wave(const DecodeArgs &a, uint32_t b, uint32_t *ring) {
    const uint64_t off = uni64(a.blk_off[b]);
    const uint32_t n = uni(a.blk_len[b]);
    uint64_t base, cap;
    record_slots<G>(a, b, off, n, base, cap);
    base = uni64(base);
    cap = uni64(cap);

    BlockReader rd;
    rd.init(ring, a.in, off, n);
    RecordStage st{};

    uint64_t kcur = 0, vcur = 0;
    if (ARENA) {
        kcur = a.arena_base ? uni64(a.arena_base[b]) : off;  // offset-addressed arenas
        vcur = kcur;
    }

    uint32_t pos = 0, nr = 0;
    int32_t status = LSM_OK;
    for (;;) {
        uint32_t rem = n - pos;
        uint32_t klen = 0, vlen = 0;
        uint64_t xval = 0;
        uint32_t vp = pos;
        if (G == LSM_GRAMMAR_V) {
            // data.go:58-76
            if (rem == 0) break;
            if (rem < 4) { status = LSM_ST_TRUNC_LEN_PREFIX; break; }
            vlen = rd.field(pos);
            if (rem - 4 < vlen) { status = LSM_ST_TRUNC_VAL; break; }
        } else if (G == LSM_GRAMMAR_KV) {
            // wal.go:107 loop of kv.go:77-115
            if (rem == 0) break;
            if (rem < 4) { status = LSM_ST_TRUNC_LEN_PREFIX; break; }
            klen = rd.field(pos);
            if (klen > kKeyCap) { status = LSM_ST_KEY_TOO_LONG; break; }
            if (rem - 4 < klen) { status = LSM_ST_TRUNC_KEY; break; }
            vp = pos + 4 + klen;
            uint32_t rem2 = n - vp;
            if (rem2 < 4) { status = LSM_ST_TRUNC_VLEN; break; }
            vlen = rd.field(vp);
            if (vlen > kValCap) { status = LSM_ST_VAL_TOO_LONG; break; }
            if (rem2 - 4 < vlen) { status = LSM_ST_TRUNC_VAL; break; }
        } else {
            // index.go:70-98
            if (rem == 0) break;
            if (rem < 4) { status = LSM_ST_IDX_OVERRUN; break; }
            klen = rd.field(pos);
            if ((uint64_t)rem < 12ull + klen) { status = LSM_ST_IDX_OVERRUN; break; }
            vp = pos + 4 + klen;
            uint32_t lo = rd.field(vp);
            uint32_t hi = rd.field(vp + 4);
            xval = (uint64_t)hi << 32 | lo;
            vlen = 8;
        }
        if (nr >= cap) { status = LSM_ST_CAPACITY; break; }

        const uint32_t slot = nr % kWave;
        st.put(slot, off + pos, klen, vlen, xval);
        if (ARENA) {
            if (G != LSM_GRAMMAR_V && a.key_arena) {
                wave_copy(rd.rsrc, rd.h + pos + 4, a.key_arena + kcur, klen);
                if (a.key_arena_off && lane_id() == 0) a.key_arena_off[base + nr] = kcur;
                kcur += klen;
            }
            if (G != LSM_GRAMMAR_IDX && a.val_arena) {
                wave_copy(rd.rsrc, rd.h + vp + 4, a.val_arena + vcur, vlen);
                if (a.val_arena_off && lane_id() == 0) a.val_arena_off[base + nr] = vcur;
                vcur += vlen;
            }
        }
        nr++;
        if (slot == kWave - 1) flush<G>(a, st, base, nr - kWave, kWave);
        pos = (G == LSM_GRAMMAR_IDX) ? vp + 8 : vp + 4 + vlen;
    }
    if (nr % kWave) flush<G>(a, st, base, nr - nr % kWave, nr % kWave);
    if (lane_id() == 0) {
        a.nrec[b] = nr;
        a.status[b] = status;
    }
}

// Speculative parallel runs (DESC mode).  After each exactly-decoded record of
// size S (key length K, value length V), all 64 lanes test the hypothesis
// "the next 64 records have the same K and V": lane i reads the length fields
// at cur + i*S (and cur + i*S + 4 + K) straight from the LDS ring.  The
// ballot's count of leading successes j is the verified run: records
// [0, j) sit exactly where predicted (each check reads the record's own
// fields), so j descriptors are stored coalesced and the cursor jumps j*S.
// The first mismatching record is re-decoded by the exact scalar step, which
// also produces the precise error status.  A block of equal-size records
// (the common LSM case) costs one exact step and one run per 64 records.
template <int G>
__device__ void decode_block_spec(const DecodeArgs &a, uint32_t b, uint32_t *ring, uint64_t off,
                                  uint32_t n, bool staged = false) {
    uint64_t base, cap;
    record_slots<G>(a, b, off, n, base, cap);
    base = uni64(base);
    cap = uni64(cap);
    const uint32_t lane = lane_id();

    BlockReader rd;
    rd.init(ring, a.in, off, n);
    if (staged) rd.hi_c = rd.nchunks < kNChunk ? rd.nchunks : kNChunk;  // DMA'd and landed
#ifdef LSM_STAMPS
    rd.ensure(rd.h);
    stamp(1);
#endif
    auto lds_u32 = [&](uint32_t p) -> uint32_t {  // per-lane read, block position p
        const uint32_t sb = rd.h + p;
        const uint32_t w = sb >> 2;
        return funnel(ring[w % kRingWords], ring[(w + 1) % kRingWords], sb);
    };

    uint32_t pos = 0, nr = 0;
    int32_t status = LSM_OK;
    for (;;) {
        // ---- exact step at pos (same checks and order as the reference) ----
        const uint32_t rem = n - pos;
        uint32_t klen = 0, vlen = 0, vp = pos;
        uint64_t xval = 0;
        if (rem == 0) break;
        if (rem < 4) {
            status = G == LSM_GRAMMAR_IDX ? LSM_ST_IDX_OVERRUN : LSM_ST_TRUNC_LEN_PREFIX;
            break;
        }
        if (G == LSM_GRAMMAR_V) {
            vlen = rd.field(pos);
            if (rem - 4 < vlen) { status = LSM_ST_TRUNC_VAL; break; }
        } else if (G == LSM_GRAMMAR_KV) {
            klen = rd.field(pos);
            if (klen > kKeyCap) { status = LSM_ST_KEY_TOO_LONG; break; }
            if (rem - 4 < klen) { status = LSM_ST_TRUNC_KEY; break; }
            vp = pos + 4 + klen;
            const uint32_t rem2 = n - vp;
            if (rem2 < 4) { status = LSM_ST_TRUNC_VLEN; break; }
            vlen = rd.field(vp);
            if (vlen > kValCap) { status = LSM_ST_VAL_TOO_LONG; break; }
            if (rem2 - 4 < vlen) { status = LSM_ST_TRUNC_VAL; break; }
        } else {
            klen = rd.field(pos);
            if ((uint64_t)rem < 12ull + klen) { status = LSM_ST_IDX_OVERRUN; break; }
            vp = pos + 4 + klen;
            xval = (uint64_t)rd.field(vp + 4) << 32 | rd.field(vp);
            vlen = 8;
        }
        if (nr >= cap) { status = LSM_ST_CAPACITY; break; }
        if (lane == 0) {
            const uint64_t ro = off + pos;
            u32x4 d;
            d.x = (uint32_t)ro;
            d.y = (uint32_t)(ro >> 32);
            d.z = klen;
            d.w = vlen;
            a.desc[base + nr] = d;
            if (G == LSM_GRAMMAR_IDX && a.idx_value) a.idx_value[base + nr] = (int64_t)xval;
        }
        nr++;
        const uint32_t S = G == LSM_GRAMMAR_V ? 4 + vlen : G == LSM_GRAMMAR_KV ? 8 + klen + vlen
                                                                              : 12 + klen;
        pos += S;

        // ---- speculative runs of records shaped like the last one ----
        for (;;) {
            if (pos >= n) break;
            rd.ensure(rd.h + pos);
            uint32_t res = rd.hi_c * kChunk;  // resident stream end
            if (res > rd.total) res = rd.total;
            const uint32_t lim = (res - rd.h) < n ? (res - rd.h) : n;
            const uint64_t pe = (uint64_t)pos + (uint64_t)(lane + 1) * S;  // record end
            const uint32_t p = pos + lane * S;
            bool ok = pe <= lim && (uint64_t)nr + lane < cap;
            uint64_t x = 0;
            if (ok) {
                if (G == LSM_GRAMMAR_V) {
                    ok = lds_u32(p) == vlen;
                } else if (G == LSM_GRAMMAR_KV) {
                    ok = (int)(lds_u32(p) == klen) & (int)(lds_u32(p + 4 + klen) == vlen);
                } else {
                    ok = lds_u32(p) == klen;
                    x = (uint64_t)lds_u32(p + 8 + klen) << 32 | lds_u32(p + 4 + klen);
                }
            }
            const uint64_t m = __ballot(ok);
            const uint32_t j = m == ~0ull ? 64u : (uint32_t)__builtin_ctzll(~m);
            if (lane < j) {
                const uint64_t ro = off + p;
                u32x4 d;
                d.x = (uint32_t)ro;
                d.y = (uint32_t)(ro >> 32);
                d.z = klen;
                d.w = vlen;
                a.desc[base + nr + lane] = d;
                if (G == LSM_GRAMMAR_IDX && a.idx_value) a.idx_value[base + nr + lane] = (int64_t)x;
            }
            nr += j;
            pos += j * S;
            if (j < 64) break;
        }
    }
    if (lane == 0) {
        a.nrec[b] = nr;
        a.status[b] = status;
    }
}

// Each wave decodes K consecutive blocks one after the other; the metadata of
// all K is fetched up front (one vector load per array), so only the block
// DMA remains on each block's critical path.
template <int G, uint32_t K, uint32_t WPG>
__global__ __launch_bounds__(64 * WPG) void decode_spec_kernel(DecodeArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t ring[WPG][kRingWords];
    const uint32_t wave = uni(threadIdx.x / kWave);
    const uint32_t b0 = uni((blockIdx.x * WPG + wave) * K);
    if (b0 >= a.nblk) return;
    const uint32_t lane = lane_id();
    uint64_t moff = 0;
    uint32_t mlen = 0;
    if (lane < K && b0 + lane < a.nblk) {
        moff = a.blk_off[b0 + lane];
        mlen = a.blk_len[b0 + lane];
    }
    stamp(0);
    for (uint32_t k = 0; k < K; k++) {
        const uint32_t b = b0 + k;
        if (b >= a.nblk) break;
        const uint64_t off = uni64((uint32_t)__builtin_amdgcn_readlane((uint32_t)moff, k) |
                                   (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(moff >> 32), k) << 32);
        const uint32_t n = __builtin_amdgcn_readlane(mlen, k);
        decode_block_spec<G>(a, b, ring[wave], off, n);
    }
    stamp(3);
}

// ---- group-per-block speculative path (DESC mode, blocks <= 4 KiB) --------
//
// A group of H lanes owns one block (64/H blocks per wave), staged whole in
// an LDS slot by LDS-DMA.  Every round each lane t of a group reads the
// length fields at pos + t*S', where S' (and K', V') is the shape of the
// group's previous record, in one batch of independent LDS reads.  Lane 0's
// position is always right; its fields are checked exactly (re-reading the
// value length when its key length differs from K') and give the shape S of
// the record at pos.  Lane t >= 1 is accepted iff S == S' and its own fields
// equal (K, V) and the record fits: then the records before it all had shape
// S and its position was right.  The group's leading run of accepted lanes
// is emitted (coalesced descriptors) and the cursor jumps.  No scalar chase:
// the control is per-lane VALU, and uniform blocks need two rounds per
// group of H records.  Oversized blocks go to the wave path afterwards.
template <int G, uint32_t H>
__global__ __launch_bounds__(64) void decode_group_kernel(DecodeArgs a) {
    constexpr uint32_t NB = kWave / H;  // blocks per wave
    constexpr uint32_t kStride = kSlotBytes + 16;
    __shared__ __attribute__((aligned(16))) uint32_t slots[NB * kStride / 4];
    const uint32_t lane = lane_id();
    const uint32_t grp = lane / H, t = lane % H;
    const uint32_t b0 = blockIdx.x * NB;
    const uint32_t b = b0 + grp;
    const bool mine = b < a.nblk;
    uint64_t off = 0;
    uint32_t n = 0;
    if (mine) {
        off = a.blk_off[b];
        n = a.blk_len[b];
    }
    const uint32_t h = (uint32_t)(off & 15);
    const bool small = mine && (uint64_t)h + n <= kSlotBytes;
    const uint64_t small_mask = __ballot(small);
    for (uint32_t j = 0; j < NB; j++) {
        if (!((small_mask >> (j * H)) & 1)) continue;
        const uint64_t offj = uni64((uint32_t)__builtin_amdgcn_readlane((uint32_t)off, j * H) |
                                    (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(off >> 32), j * H) << 32);
        const uint32_t nj = __builtin_amdgcn_readlane(n, j * H);
        const uint64_t a0 = offj & ~(uint64_t)15;
        const uint32_t tot = (uint32_t)(((offj - a0) + nj + 15) & ~(uint64_t)15);
        const rsrc_t r = make_rsrc(a.in + a0, tot);
        const uint32_t nck = (tot + kChunk - 1) / kChunk;
        for (uint32_t c = 0; c < nck; c++)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                r, (__attribute__((address_space(3))) void *)&slots[(j * kStride + c * kChunk) / 4],
                16, c * kChunk + lane * 16, 0, 0, kBlockLoadAux);
    }
    __asm__ __volatile__("s_waitcnt vmcnt(0)" ::: "memory");

    const uint32_t sbase = grp * kStride + h;
    auto rd = [&](uint32_t p) -> uint32_t {
        const uint32_t sb = sbase + p;
        const uint32_t *w = &slots[sb >> 2];
        return funnel(w[0], w[1], sb);
    };
    uint64_t base = 0, cap = 0;
    if (small) record_slots<G>(a, b, off, n, base, cap);
    const uint32_t ncap = cap < 0xFFFFFFFFull ? (uint32_t)cap : 0xFFFFFFFFu;
    const uint32_t glead = grp * H;  // group's lane 0

    bool live = small;
    int32_t status = LSM_OK;
    uint32_t pos = 0, nr = 0;
    uint32_t Kp = 0xFFFFFFFFu, Sp = 0xFFFFFFFFu;  // previous record's key length and size
    while (__ballot(live)) {
        uint32_t acc = 0, K = 0, V = 0, S = 0;
        uint64_t x = 0;
        const uint32_t p = pos + t * (Sp == 0xFFFFFFFFu ? 0u : Sp);
        const uint32_t rem = n - pos;
        if (live) {
            // speculative field reads at p (independent of each other)
            uint32_t kl = 0, vl;
            if (G == LSM_GRAMMAR_V) {
                vl = rd(p);
            } else {
                kl = rd(p);
                vl = rd(p + 4 + (Kp == 0xFFFFFFFFu ? 0u : Kp));
            }
            // lane 0: exact record at pos
            uint32_t k0 = kl, v0 = vl;
            int32_t st0 = LSM_OK;
            if (t == 0) {
                if (rem == 0) {
                    st0 = -1;  // clean end
                } else if (rem < 4) {
                    st0 = G == LSM_GRAMMAR_IDX ? LSM_ST_IDX_OVERRUN : LSM_ST_TRUNC_LEN_PREFIX;
                } else if (G == LSM_GRAMMAR_V) {
                    if (rem - 4 < v0) st0 = LSM_ST_TRUNC_VAL;
                } else if (G == LSM_GRAMMAR_KV) {
                    if (k0 > kKeyCap) st0 = LSM_ST_KEY_TOO_LONG;
                    else if (rem - 4 < k0) st0 = LSM_ST_TRUNC_KEY;
                    else {
                        const uint32_t vp = pos + 4 + k0, rem2 = n - vp;
                        if (rem2 < 4) st0 = LSM_ST_TRUNC_VLEN;
                        else {
                            if (k0 != Kp) v0 = rd(vp);
                            if (v0 > kValCap) st0 = LSM_ST_VAL_TOO_LONG;
                            else if (rem2 - 4 < v0) st0 = LSM_ST_TRUNC_VAL;
                        }
                    }
                } else {
                    if ((uint64_t)rem < 12ull + k0) st0 = LSM_ST_IDX_OVERRUN;
                }
                if (st0 == LSM_OK && nr >= ncap) st0 = LSM_ST_CAPACITY;
            }
            // broadcast lane 0's verdict and shape to its group
            st0 = __shfl(st0, glead, kWave);
            K = __shfl(k0, glead, kWave);
            V = __shfl(v0, glead, kWave);
            if (st0 != LSM_OK) {
                if (st0 > 0) status = st0;
                live = false;
            } else {
                S = G == LSM_GRAMMAR_V ? 4 + V : G == LSM_GRAMMAR_KV ? 8 + K + V : 12 + K;
                bool ok;
                if (t == 0) {
                    ok = true;
                } else {
                    ok = (S == Sp) & ((uint64_t)p + S <= n) & (nr + t < ncap);
                    if (G == LSM_GRAMMAR_V) ok = ok & (vl == V);
                    else if (G == LSM_GRAMMAR_KV) ok = ok & (kl == K) & (vl == V);
                    else ok = ok & (kl == K);
                }
                acc = ok;
                if (G == LSM_GRAMMAR_IDX && ok) x = (uint64_t)rd(p + 8 + K) << 32 | rd(p + 4 + K);
            }
        }
        // leading run of accepted lanes in each group
        const uint64_t m = __ballot(acc);
        constexpr uint64_t kGM = H == 64 ? ~0ull : ((1ull << (H % 64)) - 1);
        const uint64_t gm = (m >> glead) & kGM;
        const uint64_t inv = ~gm & kGM;
        const uint32_t j = inv ? (uint32_t)__builtin_ctzll(inv) : H;
        if (live && t < j) {
            const uint64_t ro = off + p;
            u32x4 d;
            d.x = (uint32_t)ro;
            d.y = (uint32_t)(ro >> 32);
            d.z = G == LSM_GRAMMAR_V ? 0u : K;
            d.w = G == LSM_GRAMMAR_IDX ? 8u : V;
            a.desc[base + nr + t] = d;
            if (G == LSM_GRAMMAR_IDX && a.idx_value) a.idx_value[base + nr + t] = (int64_t)x;
        }
        if (live) {
            nr += j;
            pos += j * S;
            Kp = K;
            Sp = S;
        }
    }
    if (small && t == 0) {
        a.nrec[b] = nr;
        a.status[b] = status;
    }
    // Blocks too large for a slot: wave path with slot 0 as its ring.
    const uint64_t big_mask = __ballot(mine && !small && t == 0);
    for (uint32_t j = 0; j < NB; j++)
        if ((big_mask >> (j * H)) & 1) {
            const uint32_t bb = b0 + j;
            decode_block_spec<G>(a, bb, slots, uni64(a.blk_off[bb]), uni(a.blk_len[bb]));
        }
}

template <int G, uint32_t H>
int launch_group(const DecodeArgs &a, hipStream_t s) {
    constexpr uint32_t NB = kWave / H;
    const uint32_t grid = (a.nblk + NB - 1) / NB;
    hipLaunchKernelGGL((decode_group_kernel<G, H>), dim3(grid), dim3(kWave), 0, s, a);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}

// ---- persistent, double-buffered speculative path (DESC mode, default) ----
//
// Each wave walks blocks w, w + W, w + 2W, ... (W = resident waves) with two
// 4 KiB ring slots: block k+1's four 1 KiB LDS-DMAs are issued before block k
// is decoded, and a static s_waitcnt vmcnt(4) (the four younger DMAs may stay
// in flight) releases block k.  So every wave always has a block in flight
// and the DMA latency hides behind the previous block's chase -- the
// occupancy needed for HBM rate (Little's law: ~18 blocks per CU at ~3 us)
// is reached with 20 waves per CU.  Metadata of block k+2 is prefetched with
// scalar loads.  Blocks larger than the 4 KiB ring stream on through the
// ring's own refills.
__device__ __forceinline__ void stage_block(uint32_t *ring, const uint8_t *in, uint64_t off,
                                            uint32_t n) {
    const uint64_t a0 = off & ~(uint64_t)15;
    uint64_t tot = ((off - a0) + n + 15) & ~(uint64_t)15;
    if (tot > kRingBytes) tot = kRingBytes;  // first 4 KiB; larger blocks refill later
    const rsrc_t r = make_rsrc(in + a0, (uint32_t)tot);
    const uint32_t v = lane_id() * 16;
#pragma unroll
    for (uint32_t c = 0; c < kNChunk; c++)  // always 4 ops: OOB chunks read as 0
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            r, (__attribute__((address_space(3))) void *)&ring[c * (kChunk / 4)], 16, c * kChunk + v,
            0, 0, kBlockLoadAux);
}

constexpr uint32_t kPipeWaves = 4;  // waves per workgroup (32 KiB LDS)

template <int G>
__global__ __launch_bounds__(256) void decode_pipe_kernel(DecodeArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t slots[kPipeWaves][2][kRingWords];
    const uint32_t wave = uni(threadIdx.x / kWave);
    const uint32_t W = gridDim.x * kPipeWaves;
    uint32_t b = uni(blockIdx.x * kPipeWaves + wave);
    if (b >= a.nblk) return;
    uint64_t off = uni64(a.blk_off[b]);
    uint32_t n = uni(a.blk_len[b]);
    stage_block(slots[wave][0], a.in, off, n);
    uint32_t nb = b + W;
    uint64_t noff = 0;
    uint32_t nn = 0;
    if (nb < a.nblk) {
        noff = uni64(a.blk_off[nb]);
        nn = uni(a.blk_len[nb]);
    }
    for (uint32_t k = 0;; k++) {
        uint32_t *cur = slots[wave][k & 1];
        const bool more = nb < a.nblk;
        if (more) {
            stage_block(slots[wave][(k + 1) & 1], a.in, noff, nn);
            __asm__ __volatile__("s_waitcnt vmcnt(4)" ::: "memory");
        } else {
            __asm__ __volatile__("s_waitcnt vmcnt(0)" ::: "memory");
        }
        // prefetch metadata two blocks ahead
        const uint32_t nnb = nb + W;
        uint64_t poff = 0;
        uint32_t pn = 0;
        if (more && nnb < a.nblk) {
            poff = uni64(a.blk_off[nnb]);
            pn = uni(a.blk_len[nnb]);
        }
        decode_block_spec<G>(a, b, cur, off, n, true);
        if (!more) break;
        b = nb;
        off = noff;
        n = nn;
        nb = nnb;
        noff = poff;
        nn = pn;
    }
}

template <int G>
int launch_pipe(lsm_ctx *ctx, const DecodeArgs &a, hipStream_t s) {
    // 5 workgroups (20 waves) per CU fit the LDS; a fixed residency-sized grid.
    const uint32_t cus = ctx ? (uint32_t)lsm_ctx_num_cus(ctx) : 256u;
    const uint32_t want = cus * 5;
    const uint32_t need = (a.nblk + kPipeWaves - 1) / kPipeWaves;
    const uint32_t grid = need < want ? need : want;
    hipLaunchKernelGGL((decode_pipe_kernel<G>), dim3(grid), dim3(kWave * kPipeWaves), 0, s, a);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}

template <int G, uint32_t K, uint32_t WPG = kWavesPerWG>
int launch_spec(const DecodeArgs &a, hipStream_t s) {
    const uint32_t waves = (a.nblk + K - 1) / K;
    const uint32_t grid = (waves + WPG - 1) / WPG;
    hipLaunchKernelGGL((decode_spec_kernel<G, K, WPG>), dim3(grid), dim3(kWave * WPG), 0, s, a);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}

template <int G, bool ARENA>
__global__ __launch_bounds__(256) void decode_blocks_kernel(DecodeArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t ring[kWavesPerWG][kRingWords];
    const uint32_t wave = uni(threadIdx.x / kWave);
    const uint32_t b = uni(blockIdx.x * kWavesPerWG + wave);
    if (b >= a.nblk) return;
    decode_block_wave<G, ARENA>(a, b, ring[wave]);
}

// ---- lane-per-block path (DESC mode) ----------------------------------------
//
// The record chain is serial inside a block, so a wave-uniform chase is bound
// by the CU's single scalar unit (~1 instruction/cycle/CU).  Here each lane
// chases its own block instead: a one-wave workgroup owns kLaneBlocks blocks,
// LDS-DMAs each (<= 4 KiB + alignment) into a private slot with four
// coalesced 1 KiB loads, then every lane walks its block's length fields with
// per-lane unaligned LDS reads (two ds_read_b32 + v_alignbyte per field) and
// writes its descriptors.  Slots are skewed by 16 bytes so lanes walking
// identically laid out blocks hit different banks.  Blocks that do not fit a
// slot are decoded afterwards by the wave path.

template <int G, uint32_t kLaneBlocks>
__global__ __launch_bounds__(64) void decode_lanes_kernel(DecodeArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t slots[kLaneBlocks * kSlotStride / 4];
    stamp(0);
    const uint32_t lane = lane_id();
    const uint32_t b0 = blockIdx.x * kLaneBlocks;
    const uint32_t b = b0 + lane;
    const bool mine = lane < kLaneBlocks && b < a.nblk;
    uint64_t off = 0;
    uint32_t n = 0;
    if (mine) {
        off = a.blk_off[b];
        n = a.blk_len[b];
    }
    const uint32_t h = (uint32_t)(off & 15);
    const bool small = mine && (uint64_t)h + n <= kSlotBytes;
    const uint64_t small_mask = __ballot(small);

    // Stage every small block into its slot: 4 x 1 KiB LDS-DMA per block.
    for (uint32_t j = 0; j < kLaneBlocks; j++) {
        if (!((small_mask >> j) & 1)) continue;
        const uint64_t offj = uni64(__shfl(off, j, kWave));
        const uint32_t nj = uni(__shfl(n, j, kWave));
        const uint64_t a0 = offj & ~(uint64_t)15;
        const uint32_t tot = (uint32_t)(((offj - a0) + nj + 15) & ~(uint64_t)15);
        const rsrc_t r = make_rsrc(a.in + a0, tot);
        const uint32_t nck = (tot + kChunk - 1) / kChunk;
        for (uint32_t c = 0; c < nck; c++)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                r, (__attribute__((address_space(3))) void *)&slots[(j * kSlotStride + c * kChunk) / 4],
                16, c * kChunk + lane * 16, 0, 0, kBlockLoadAux);
    }
    __asm__ __volatile__("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(1);

    if (small) {
        // Byte address of this lane's slot; reads past the slot return
        // another slot's bytes or 0 (LDS bounds) and are never accepted.
        const uint32_t sbase = lane * kSlotStride + h;
        auto rd = [&](uint32_t p) -> uint32_t {
            const uint32_t sb = sbase + p;
            const uint32_t *w = &slots[sb >> 2];
            return funnel(w[0], w[1], sb);
        };
        uint64_t base, cap;
        record_slots<G>(a, b, off, n, base, cap);
        u32x4 *dp = a.desc + base;
        int64_t *xp = a.idx_value ? a.idx_value + base : nullptr;
        const uint32_t ncap = cap < 0xFFFFFFFFull ? (uint32_t)cap : 0xFFFFFFFFu;
        uint32_t pos = 0, nr = 0;
        // Straight-line record step; a failing check ends the lane's loop and
        // the (rare) status is resolved once afterwards from pos.
        for (;;) {
            const uint32_t rem = n - pos;
            uint32_t klen = 0, vlen, vp = pos, nxt;
            bool ok;
            if (G == LSM_GRAMMAR_V) {
                vlen = rd(pos);
                ok = (rem >= 4) & (rem - 4 >= vlen);
                nxt = pos + 4 + vlen;
            } else if (G == LSM_GRAMMAR_KV) {
                klen = rd(pos);
                vp = pos + 4 + klen;
                vlen = rd(vp);
                const uint32_t rem2 = n - vp;
                ok = (rem >= 4) & (klen <= kKeyCap) & (rem - 4 >= klen) & (rem2 >= 4) &
                     (vlen <= kValCap) & (rem2 - 4 >= vlen);
                nxt = vp + 4 + vlen;
            } else {
                klen = rd(pos);
                vp = pos + 4 + klen;
                vlen = 8;
                ok = (rem >= 12) & (rem - 12 >= klen);
                nxt = vp + 8;
            }
            ok = ok & (nr < ncap);
            if (!ok) break;
            const uint64_t ro = off + pos;
            u32x4 d;
            d.x = (uint32_t)ro;
            d.y = (uint32_t)(ro >> 32);
            d.z = klen;
            d.w = vlen;
            dp[nr] = d;
            if (G == LSM_GRAMMAR_IDX && xp) xp[nr] = (int64_t)((uint64_t)rd(vp + 4) << 32 | rd(vp));
            nr++;
            pos = nxt;
        }
        // Status of the stop at pos (same precedence as the reference).
        int32_t status = LSM_OK;
        const uint32_t rem = n - pos;
        if (rem != 0) {
            if (G == LSM_GRAMMAR_V) {
                status = rem < 4 ? LSM_ST_TRUNC_LEN_PREFIX
                       : rem - 4 < rd(pos) ? LSM_ST_TRUNC_VAL : LSM_ST_CAPACITY;
            } else if (G == LSM_GRAMMAR_KV) {
                if (rem < 4) status = LSM_ST_TRUNC_LEN_PREFIX;
                else {
                    const uint32_t klen = rd(pos);
                    if (klen > kKeyCap) status = LSM_ST_KEY_TOO_LONG;
                    else if (rem - 4 < klen) status = LSM_ST_TRUNC_KEY;
                    else {
                        const uint32_t vp = pos + 4 + klen, rem2 = n - vp;
                        const uint32_t vlen = rem2 >= 4 ? rd(vp) : 0;
                        status = rem2 < 4 ? LSM_ST_TRUNC_VLEN
                               : vlen > kValCap ? LSM_ST_VAL_TOO_LONG
                               : rem2 - 4 < vlen ? LSM_ST_TRUNC_VAL : LSM_ST_CAPACITY;
                    }
                }
            } else {
                status = (rem < 12 || rem - 12 < rd(pos)) ? LSM_ST_IDX_OVERRUN : LSM_ST_CAPACITY;
            }
        }
        a.nrec[b] = nr;
        a.status[b] = status;
    }

    stamp(2);
    // Blocks too large for a slot: whole-wave streaming path, slot 0 as ring.
    const uint64_t big_mask = __ballot(mine && !small);
    for (uint32_t j = 0; j < kLaneBlocks; j++)
        if ((big_mask >> j) & 1) decode_block_wave<G, false>(a, b0 + j, slots);
    stamp(3);
}

// ---- planning: exclusive scans over per-block quantities -----------------

constexpr uint32_t kScanThreads = 256;
constexpr uint32_t kScanPer = 16;
constexpr uint32_t kScanTile = kScanThreads * kScanPer;

__device__ __forceinline__ uint64_t plan_value(int mode, uint32_t len) {
    switch (mode) {
    case 0: return len / 4;   // V
    case 1: return len / 8;   // KV
    case 2: return len / 12;  // IDX
    default: return len;      // arena bytes
    }
}

__device__ uint64_t block_excl_scan(uint64_t v, uint64_t *total) {
    __shared__ uint64_t wsum[kScanThreads / kWave];
    uint64_t wt;
    uint64_t x = wave_excl_scan64(v, &wt);
    uint32_t w = threadIdx.x / kWave;
    if (lane_id() == 0) wsum[w] = wt;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
    for (uint32_t i = 0; i < kScanThreads / kWave; i++) {
        if (i < w) pre += wsum[i];
        tot += wsum[i];
    }
    __syncthreads();
    *total = tot;
    return x + pre;
}

__global__ __launch_bounds__(kScanThreads) void plan_tile_sums(int mode, const uint32_t *len,
                                                               uint32_t n, uint64_t *partial) {
    uint64_t s = 0;
    uint64_t i0 = (uint64_t)blockIdx.x * kScanTile + threadIdx.x * kScanPer;
    for (uint32_t j = 0; j < kScanPer; j++)
        if (i0 + j < n) s += plan_value(mode, len[i0 + j]);
    uint64_t tot;
    block_excl_scan(s, &tot);
    if (threadIdx.x == 0) partial[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kScanThreads) void plan_scan_partials(uint64_t *partial,
                                                                   uint32_t ntiles, uint64_t *out,
                                                                   uint32_t n) {
    uint64_t carry = 0;
    for (uint32_t t0 = 0; t0 < ntiles; t0 += kScanThreads) {
        uint32_t t = t0 + threadIdx.x;
        uint64_t v = t < ntiles ? partial[t] : 0;
        uint64_t tot;
        uint64_t x = block_excl_scan(v, &tot);
        if (t < ntiles) partial[t] = carry + x;
        carry += tot;
    }
    if (threadIdx.x == 0) out[n] = carry;
}

__global__ __launch_bounds__(kScanThreads) void plan_tile_apply(int mode, const uint32_t *len,
                                                                uint32_t n,
                                                                const uint64_t *partial,
                                                                uint64_t *out) {
    uint64_t vals[kScanPer];
    uint64_t s = 0;
    uint64_t i0 = (uint64_t)blockIdx.x * kScanTile + threadIdx.x * kScanPer;
    for (uint32_t j = 0; j < kScanPer; j++) {
        vals[j] = (i0 + j < n) ? plan_value(mode, len[i0 + j]) : 0;
        s += vals[j];
    }
    uint64_t tot;
    uint64_t pre = block_excl_scan(s, &tot) + partial[blockIdx.x];
    for (uint32_t j = 0; j < kScanPer; j++) {
        if (i0 + j < n) out[i0 + j] = pre;
        pre += vals[j];
    }
}

int plan_scan(int mode, const uint32_t *d_len, uint32_t n, uint64_t *d_out, void *ws,
              size_t ws_bytes, hipStream_t s) {
    uint32_t ntiles = (n + kScanTile - 1) / kScanTile;
    if (ntiles == 0) ntiles = 1;
    if (ws_bytes < (size_t)ntiles * 8 || (!ws && n)) return LSM_ESPACE;
    uint64_t *partial = static_cast<uint64_t *>(ws);
    if (n == 0) {
        LSM_HIP_CHECK(hipMemsetAsync(d_out, 0, 8, s));
        return 0;
    }
    hipLaunchKernelGGL(plan_tile_sums, dim3(ntiles), dim3(kScanThreads), 0, s, mode, d_len, n,
                       partial);
    hipLaunchKernelGGL(plan_scan_partials, dim3(1), dim3(kScanThreads), 0, s, partial, ntiles,
                       d_out, n);
    hipLaunchKernelGGL(plan_tile_apply, dim3(ntiles), dim3(kScanThreads), 0, s, mode, d_len, n,
                       partial, d_out);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}

// ---- streaming lane-per-block path (DESC mode, default) ------------------
//
// Each lane owns one block of any size and chases it through a per-wave LDS
// ring of W rows; row r holds stream bytes [16r, 16r+16) of every lane's own
// block, gathered by ONE global_load_lds_dwordx4 per row (per-lane source
// address, lane L's 16 bytes land at row + 16L).  A round refills rows
// [r_lo, r_lo + W) (r_lo = the lowest row any lane still needs), waits once,
// then every lane consumes as many length fields as the window holds.  The
// chase is a field-granular state machine so one long key never stalls the
// window, and rows that every lane has jumped over are never loaded.
template <int G, uint32_t BL, uint32_t W>
__global__ __launch_bounds__(64) void decode_stream_kernel(DecodeArgs a) {
    constexpr uint32_t kRow = BL * 16;  // bytes per ring row
    __shared__ __attribute__((aligned(16))) uint32_t ring[W * kRow / 4];
    stamp(0);
    const uint32_t lane = lane_id();
    const uint32_t b = blockIdx.x * BL + lane;
    const bool mine = lane < BL && b < a.nblk;
    uint64_t off = 0;
    uint32_t n = 0;
    if (mine) {
        off = a.blk_off[b];
        n = a.blk_len[b];
    }
    const uint64_t a0 = off & ~(uint64_t)15;
    const uint32_t h = (uint32_t)(off - a0);
    const uint8_t *g = a.in + a0;
    const uint32_t rows = (uint32_t)(((uint64_t)h + n + 15) / 16);
    uint64_t base = 0, cap = 0;
    if (mine) record_slots<G>(a, b, off, n, base, cap);
    u32x4 *dp = a.desc + base;
    int64_t *xp = (G == LSM_GRAMMAR_IDX && a.idx_value) ? a.idx_value + base : nullptr;
    const uint32_t ncap = cap < 0xFFFFFFFFull ? (uint32_t)cap : 0xFFFFFFFFu;

    const uint32_t lane_w = lane * 4;  // this lane's dword inside a row
    auto dword = [&](uint32_t i) -> uint32_t {  // stream dword i of this lane
        return ring[((i >> 2) % W) * (kRow / 4) + lane_w + (i & 3)];
    };

    bool active = mine;
    int32_t status = LSM_OK;
    uint32_t pos = 0, vp = 0, klen = 0, phase = 0, nr = 0;
    uint32_t r_lo = 0, r_loaded = 0;
    for (;;) {
        // Refill rows [max(r_loaded, r_lo), r_lo + W): one gather per row.
        const uint32_t r1 = r_lo + W;
        for (uint32_t r = r_loaded > r_lo ? r_loaded : r_lo; r < r1; r++) {
            if (active && r < rows)
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)(g + 16 * (uint64_t)r),
                    (__attribute__((address_space(3))) void *)&ring[(r % W) * (kRow / 4)], 16, 0, 0);
        }
        r_loaded = r1;
        __asm__ __volatile__("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t win_end = 16 * r1;

        // Consume every field the window holds.
        while (active) {
            const uint32_t fp = phase ? vp : pos;
            const uint32_t rem = n - fp;
            if (phase == 0 && rem == 0) { active = false; break; }  // clean end
            const uint32_t need = (G == LSM_GRAMMAR_IDX && phase) ? 8 : 4;
            if (rem < need) {
                status = G == LSM_GRAMMAR_IDX ? LSM_ST_IDX_OVERRUN
                       : phase ? LSM_ST_TRUNC_VLEN : LSM_ST_TRUNC_LEN_PREFIX;
                active = false;
                break;
            }
            const uint32_t sb = h + fp;
            if (sb + need > win_end) break;  // next round
            const uint32_t i = sb >> 2;
            const uint32_t d0 = dword(i), d1 = dword(i + 1);
            const uint32_t f = funnel(d0, d1, sb);
            if (phase == 0 && G != LSM_GRAMMAR_V) {
                klen = f;
                if (G == LSM_GRAMMAR_KV) {
                    if (klen > kKeyCap) { status = LSM_ST_KEY_TOO_LONG; active = false; break; }
                    if (rem - 4 < klen) { status = LSM_ST_TRUNC_KEY; active = false; break; }
                } else if ((uint64_t)rem < 12ull + klen) {
                    status = LSM_ST_IDX_OVERRUN;
                    active = false;
                    break;
                }
                vp = pos + 4 + klen;
                phase = 1;
                continue;
            }
            // value length (V, KV) or index offset (IDX): the record is complete
            uint32_t vlen;
            uint64_t xval = 0;
            if (G == LSM_GRAMMAR_IDX) {
                xval = (uint64_t)funnel(d1, dword(i + 2), sb) << 32 | f;
                vlen = 8;
            } else {
                vlen = f;
                if (G == LSM_GRAMMAR_KV && vlen > kValCap) { status = LSM_ST_VAL_TOO_LONG; active = false; break; }
                if (rem - 4 < vlen) { status = LSM_ST_TRUNC_VAL; active = false; break; }
            }
            if (nr >= ncap) { status = LSM_ST_CAPACITY; active = false; break; }
            const uint64_t ro = off + pos;
            u32x4 d;
            d.x = (uint32_t)ro;
            d.y = (uint32_t)(ro >> 32);
            d.z = G == LSM_GRAMMAR_V ? 0u : klen;
            d.w = vlen;
            dp[nr] = d;
            if (G == LSM_GRAMMAR_IDX && xp) xp[nr] = (int64_t)xval;
            nr++;
            const uint32_t rs = G == LSM_GRAMMAR_V ? pos : vp;
            pos = G == LSM_GRAMMAR_IDX ? rs + 8 : rs + 4 + vlen;
            phase = 0;
        }
        // Lowest row any lane still needs; all lanes done -> exit.
        uint32_t need_row = active ? (h + (phase ? vp : pos)) >> 4 : 0xFFFFFFFFu;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const uint32_t o = __shfl_xor(need_row, d, kWave);
            need_row = o < need_row ? o : need_row;
        }
        r_lo = uni(need_row);
        if (r_lo == 0xFFFFFFFFu) break;
    }
    stamp(2);
    if (mine) {
        a.nrec[b] = nr;
        a.status[b] = status;
    }
    stamp(3);
}

template <int G, uint32_t BL, uint32_t W>
int launch_stream(const DecodeArgs &a, hipStream_t s) {
    uint32_t grid = (a.nblk + BL - 1) / BL;
    hipLaunchKernelGGL((decode_stream_kernel<G, BL, W>), dim3(grid), dim3(kWave), 0, s, a);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}

template <int G, uint32_t B>
int launch_lanes(const DecodeArgs &a, hipStream_t s) {
    uint32_t grid = (a.nblk + B - 1) / B;
    hipLaunchKernelGGL((decode_lanes_kernel<G, B>), dim3(grid), dim3(kWave), 0, s, a);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}

template <int G, bool ARENA>
int launch_decode(lsm_ctx *ctx, const DecodeArgs &a, hipStream_t s) {
    if (!ARENA) {
        // Default: wave-per-block with speculative parallel runs, one wave per
        // workgroup (finer dispatch/retire granularity than 4-wave groups:
        // 4413 vs 4250 GiB/s on decode4k with nt loads, same box).
        // LSM_DECODE_KERNEL selects variants for A/B measurement.
        static const int variant = [] {
            const char *e = getenv("LSM_DECODE_KERNEL");
            if (!e) return 0;
            if (!strcmp(e, "stream64x16")) return 1;
            if (!strcmp(e, "stream32x64")) return 2;
            if (!strcmp(e, "stream64x32")) return 3;
            if (!strcmp(e, "lanes")) return 9;
            if (!strcmp(e, "stream32x32")) return 4;
            if (!strcmp(e, "spec4")) return 10;
            if (!strcmp(e, "spec")) return 30;
            if (!strcmp(e, "spec_w1")) return 31;
            if (!strcmp(e, "spec_w2")) return 32;
            if (!strcmp(e, "pipe")) return 33;
            if (!strcmp(e, "group64")) return 20;
            if (!strcmp(e, "group32")) return 21;
            if (!strcmp(e, "group16")) return 22;
            if (!strcmp(e, "spec2")) return 11;
            if (!strcmp(e, "spec8")) return 12;
            if (!strcmp(e, "spec16")) return 13;
            return 0;
        }();
        switch (variant) {
        case 0: return launch_spec<G, 1, 1>(a, s);  // one-wave workgroups: measured best
        case 33: return launch_pipe<G>(ctx, a, s);
        case 30: return launch_spec<G, 1>(a, s);
        case 31: return launch_spec<G, 1, 1>(a, s);
        case 32: return launch_spec<G, 1, 2>(a, s);
        case 20: return launch_group<G, 64>(a, s);
        case 21: return launch_group<G, 32>(a, s);
        case 22: return launch_group<G, 16>(a, s);
        case 10: return launch_spec<G, 4>(a, s);
        case 11: return launch_spec<G, 2>(a, s);
        case 12: return launch_spec<G, 8>(a, s);
        case 13: return launch_spec<G, 16>(a, s);
        case 4: return launch_stream<G, 32, 32>(a, s);
        case 1: return launch_stream<G, 64, 16>(a, s);
        case 2: return launch_stream<G, 32, 64>(a, s);
        case 3: return launch_stream<G, 64, 32>(a, s);
        case 9: break;
        default: return launch_stream<G, 32, 32>(a, s);
        }
        // Blocks per wave (LDS slots): 3 admits 13 one-wave workgroups per CU.
        static const int lb = [] {
            const char *e = getenv("LSM_LANE_BLOCKS");
            return e ? atoi(e) : 3;
        }();
        switch (lb) {
        case 3: return launch_lanes<G, 3>(a, s);
        case 4: return launch_lanes<G, 4>(a, s);
        case 8: return launch_lanes<G, 8>(a, s);
        case 15: return launch_lanes<G, 15>(a, s);
        case 7: return launch_lanes<G, 7>(a, s);
        default: return launch_lanes<G, 3>(a, s);
        }
    } else {
        uint32_t grid = (a.nblk + kWavesPerWG - 1) / kWavesPerWG;
        hipLaunchKernelGGL((decode_blocks_kernel<G, ARENA>), dim3(grid),
                           dim3(kWave * kWavesPerWG), 0, s, a);
    }
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace
}  // namespace lsm

using namespace lsm;

extern "C" uint64_t lsm_max_records(int grammar, uint64_t len) {
    switch (grammar) {
    case LSM_GRAMMAR_V: return len / 4;
    case LSM_GRAMMAR_KV: return len / 8;
    case LSM_GRAMMAR_IDX: return len / 12;
    default: return 0;
    }
}

extern "C" size_t lsm_plan_workspace_bytes(uint32_t nblk) {
    size_t ntiles = (nblk + kScanTile - 1) / kScanTile;
    return (ntiles ? ntiles : 1) * 8;
}

extern "C" int lsm_plan_rec_base(lsm_ctx *ctx, int grammar, const uint32_t *d_blk_len,
                                 uint32_t nblk, uint64_t *d_rec_base, void *d_workspace,
                                 size_t ws_bytes, void *stream) {
    if (!ctx || !d_rec_base || (nblk && !d_blk_len)) return LSM_EINVAL;
    if (grammar < LSM_GRAMMAR_V || grammar > LSM_GRAMMAR_IDX) return LSM_EINVAL;
    int mode = grammar == LSM_GRAMMAR_V ? 0 : grammar == LSM_GRAMMAR_KV ? 1 : 2;
    return plan_scan(mode, d_blk_len, nblk, d_rec_base, d_workspace, ws_bytes,
                     static_cast<hipStream_t>(stream));
}

extern "C" int lsm_plan_arena_base(lsm_ctx *ctx, const uint32_t *d_blk_len, uint32_t nblk,
                                   uint64_t *d_arena_base, void *d_workspace, size_t ws_bytes,
                                   void *stream) {
    if (!ctx || !d_arena_base || (nblk && !d_blk_len)) return LSM_EINVAL;
    return plan_scan(3, d_blk_len, nblk, d_arena_base, d_workspace, ws_bytes,
                     static_cast<hipStream_t>(stream));
}

// ---- compaction: decoded records -> one dense array -----------------------
//
// The decode writes block b's records at its capacity slots (rec_base or
// offset-addressed), so the per-record arrays are sparse.  A consumer on the
// host (or the next stage) wants them dense: out_base = exclusive scan of
// nrec (plan_scan), then one wave per block copies its nrec descriptors
// (16 B per lane, coalesced) and IDX values.
__global__ __launch_bounds__(256) void compact_kernel(int grammar, const uint64_t *blk_off,
                                                      uint32_t nblk, const u32x4 *desc,
                                                      const int64_t *idx, const uint64_t *rec_base,
                                                      const uint32_t *nrec, const uint64_t *out_base,
                                                      u32x4 *dense, int64_t *dense_idx) {
    const uint32_t b = uni(blockIdx.x * 4 + threadIdx.x / kWave);
    if (b >= nblk) return;
    const uint32_t R = grammar == LSM_GRAMMAR_V ? 4 : grammar == LSM_GRAMMAR_KV ? 8 : 12;
    const uint64_t src = rec_base ? uni64(rec_base[b]) : uni64(blk_off[b]) / R;
    const uint64_t dst = uni64(out_base[b]);
    const uint32_t n = uni(nrec[b]);
    for (uint32_t i = lane_id(); i < n; i += kWave) {
        dense[dst + i] = __builtin_nontemporal_load(&desc[src + i]);
        if (dense_idx) dense_idx[dst + i] = idx[src + i];
    }
}

extern "C" int lsm_compact_records(lsm_ctx *ctx, int grammar, const uint64_t *d_blk_off,
                                   uint32_t nblk, const lsm_decode_out *out, lsm_rec_desc *d_dense,
                                   int64_t *d_dense_idx, uint64_t *d_dense_base, void *d_workspace,
                                   size_t ws_bytes, void *stream) {
    if (!ctx || !out || !d_dense_base) return LSM_EINVAL;
    if (grammar < LSM_GRAMMAR_V || grammar > LSM_GRAMMAR_IDX) return LSM_EINVAL;
    if (nblk && (!out->desc || !out->nrec || !d_dense || (!out->rec_base && !d_blk_off)))
        return LSM_EINVAL;
    if (d_dense_idx && (grammar != LSM_GRAMMAR_IDX || !out->idx_value)) return LSM_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int rc = plan_scan(3, out->nrec, nblk, d_dense_base, d_workspace, ws_bytes, s);
    if (rc) return rc;
    if (nblk == 0) return 0;
    hipLaunchKernelGGL(compact_kernel, dim3((nblk + 3) / 4), dim3(256), 0, s, grammar, d_blk_off,
                       nblk, reinterpret_cast<const u32x4 *>(out->desc), out->idx_value,
                       out->rec_base, out->nrec, d_dense_base, reinterpret_cast<u32x4 *>(d_dense),
                       d_dense_idx);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}

extern "C" int lsm_decode_blocks(lsm_ctx *ctx, int grammar, const uint8_t *d_in,
                                 const uint64_t *d_blk_off, const uint32_t *d_blk_len,
                                 uint32_t nblk, const lsm_decode_out *out, void *stream) {
    if (!ctx || !out) return LSM_EINVAL;
    if (nblk == 0) return 0;
    if (!d_in || !d_blk_off || !d_blk_len || !out->desc || !out->nrec || !out->status)
        return LSM_EINVAL;
    if (grammar < LSM_GRAMMAR_V || grammar > LSM_GRAMMAR_IDX) return LSM_EINVAL;
    bool arena = out->key_arena || out->val_arena;
    DecodeArgs a;
    a.in = d_in;
    a.blk_off = d_blk_off;
    a.blk_len = d_blk_len;
    a.nblk = nblk;
    a.desc = reinterpret_cast<u32x4 *>(out->desc);
    a.rec_base = out->rec_base;
    a.nrec = out->nrec;
    a.status = out->status;
    a.idx_value = out->idx_value;
    a.key_arena = out->key_arena;
    a.val_arena = out->val_arena;
    a.arena_base = out->arena_base;
    a.key_arena_off = out->key_arena_off;
    a.val_arena_off = out->val_arena_off;
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (grammar) {
    case LSM_GRAMMAR_V: return arena ? launch_decode<LSM_GRAMMAR_V, true>(ctx, a, s)
                                     : launch_decode<LSM_GRAMMAR_V, false>(ctx, a, s);
    case LSM_GRAMMAR_KV: return arena ? launch_decode<LSM_GRAMMAR_KV, true>(ctx, a, s)
                                      : launch_decode<LSM_GRAMMAR_KV, false>(ctx, a, s);
    default: return arena ? launch_decode<LSM_GRAMMAR_IDX, true>(ctx, a, s)
                          : launch_decode<LSM_GRAMMAR_IDX, false>(ctx, a, s);
    }
}

#ifdef LSM_STAMPS
extern "C" int lsm_debug_set_stamps(void *d_buf) {
    LSM_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(lsm::g_stamps), &d_buf, sizeof(void *)));
    return 0;
}
#endif
