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
    uint32_t split;  // 1: blocks larger than the 4 KiB ring are left to decode_large_kernel
    uint32_t dbg;    // diagnostics only (LSM_DECODE_DBG): bit 0 no speculative runs,
                     // bit 2 stop after one record, bit 3 global verification of
                     // streamed uniform blocks (A/B; off by default)
};

// Streams one block through this wave's LDS ring and serves u32 length
// fields at wave-uniform block positions.
//
// Ring: NCH x 1 KiB chunks, filled by LDS-DMA (buffer_load_dwordx4 ... lds:
// no VGPR staging).  Window: each lane holds 16 raw bytes of a 1 KiB, 16-byte
// aligned slice of the stream (one ds_read_b128); a field at stream byte s is
// two v_readlane of the lanes/dwords covering [s, s+4) plus a scalar funnel
// shift, so a 4 KiB block costs ~5 LDS round trips instead of one per record.
// NCH = 4 (4 KiB) for blocks that fit whole; blocks larger than that stream
// through a 16 KiB ring (decode_large_kernel) with up to 15 KiB in flight.
template <int N>
__device__ __forceinline__ void wait_vmcnt_le(uint32_t k) {
    // s_waitcnt takes an immediate: one arm per count (N <= 16).
#define LSM_VMW(i) case i: __asm__ __volatile__("s_waitcnt vmcnt(" #i ")" ::: "memory"); break;
    switch (k < N ? k : N - 1) {
    LSM_VMW(0) LSM_VMW(1) LSM_VMW(2) LSM_VMW(3) LSM_VMW(4) LSM_VMW(5) LSM_VMW(6) LSM_VMW(7)
    LSM_VMW(8) LSM_VMW(9) LSM_VMW(10) LSM_VMW(11) LSM_VMW(12) LSM_VMW(13) LSM_VMW(14)
    default: __asm__ __volatile__("s_waitcnt vmcnt(15)" ::: "memory"); break;
    }
#undef LSM_VMW
}

template <uint32_t NCH>
struct BlockReaderT {
    static constexpr uint32_t kBytes = NCH * kChunk;
    uint32_t *ring;
    rsrc_t rsrc;
    uint32_t h;        // block start inside its first 16-byte line
    uint32_t total;    // loadable stream bytes: round_up16(h + n)
    uint32_t nchunks;  // chunks covering [0, total)
    uint32_t hi_c;     // chunks [.., hi_c) have been issued into the ring
    uint32_t landed;   // chunks [.., landed) are known to be in LDS
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
        landed = 0;
        have_win = false;
        wb = 0;
    }

    // Make stream bytes [s0, s0 + want) resident (clamped to the block and
    // to the ring's reach from s0's chunk).  Every free ring slot is refilled,
    // but the wait is counted: only the chunks asked for must have landed, the
    // younger ones stay in flight while the chase runs.  vmcnt retires in
    // issue order across loads, stores and LDS-DMA, so descriptor stores
    // issued after a prefetch only make the count conservative.  (A plain
    // vmcnt(0) here streams a block larger than the ring at one HBM round
    // trip per refill.)
    __device__ __forceinline__ void ensure(uint32_t s0, uint32_t want = kChunk) {
        const uint32_t c0 = s0 / kChunk;
        // Top up: every slot whose chunk lies behind s0 is free; refill it now
        // (even when the bytes asked for are already resident), so a chunk is
        // issued NCH - 1 chunks before the chase reaches it.
        uint32_t last = c0 + NCH;
        if (last > nchunks) last = nchunks;
        if (last > hi_c) {
            const uint32_t voff = lane_id() * 16;
            for (uint32_t c = hi_c > c0 ? hi_c : c0; c < last; c++)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rsrc, (__attribute__((address_space(3))) void *)&ring[(c % NCH) * (kChunk / 4)],
                    16, voff + c * kChunk, 0, 0, kBlockLoadAux);
            hi_c = last;
        }
        uint64_t need_end = (uint64_t)s0 + want;
        if (need_end > total) need_end = total;
        if (need_end > (uint64_t)last * kChunk) need_end = (uint64_t)last * kChunk;
        const uint32_t need_hi = (uint32_t)((need_end + kChunk - 1) / kChunk);
        if (need_hi <= landed) return;
        // The DMA writes are invisible to the compiler's waitcnt tracking of
        // ds_read; wait for them explicitly before any LDS read of them.
        wait_vmcnt_le<NCH>(hi_c - need_hi);
        landed = need_hi;
    }

    __device__ __forceinline__ void load_window(uint32_t s) {
        wb = s & ~15u;
        ensure(wb);
        const uint32_t w = ((wb + lane_id() * 16) % kBytes) / 4;
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
using BlockReader = BlockReaderT<kNChunk>;

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
template <int G, uint32_t NCH = kNChunk>
__device__ void decode_block_spec(const DecodeArgs &a, uint32_t b, uint32_t *ring, uint64_t off,
                                  uint32_t n, bool staged = false) {
    constexpr uint32_t kWords = NCH * kChunk / 4;
    uint64_t base, cap;
    record_slots<G>(a, b, off, n, base, cap);
    base = uni64(base);
    cap = uni64(cap);
    const uint32_t lane = lane_id();

    BlockReaderT<NCH> rd;
    rd.init(ring, a.in, off, n);
    if (staged) rd.hi_c = rd.landed = rd.nchunks < NCH ? rd.nchunks : NCH;  // DMA'd and landed
#ifdef LSM_STAMPS
    rd.ensure(rd.h);
    stamp(1);
#endif
    auto lds_u32 = [&](uint32_t p) -> uint32_t {  // per-lane read, block position p
        const uint32_t sb = rd.h + p;
        const uint32_t w = sb >> 2;
        return funnel(ring[w % kWords], ring[(w + 1) % kWords], sb);
    };

    // Wave-uniform field at block position p: two LDS dwords (a broadcast
    // read), a funnel shift and one readfirstlane.  The bytes must be landed.
    auto ufield = [&](uint32_t p) -> uint32_t {
        const uint32_t sb = rd.h + p;
        const uint32_t w = sb >> 2;
        return uni(funnel(ring[w % kWords], ring[(w + 1) % kWords], sb));
    };

    // Exact-step records are staged one per lane and stored 64 at a time: a
    // store between a ring refill and its counted wait is younger than the
    // chunks in flight, so one store per record would make every wait drain
    // the whole prefetch (vmcnt counts stores too).  Staged records occupy
    // consecutive slots s_first.. (the stage is flushed before a run).
    uint32_t s_pos = 0, s_k = 0, s_v = 0, s_xlo = 0, s_xhi = 0, ns = 0, s_first = 0;
    auto flush_stage = [&]() {
        if (ns && lane < ns) {
            const uint64_t ro = off + s_pos;
            u32x4 d;
            d.x = (uint32_t)ro;
            d.y = (uint32_t)(ro >> 32);
            d.z = s_k;
            d.w = s_v;
            a.desc[base + s_first + lane] = d;
            if (G == LSM_GRAMMAR_IDX && a.idx_value)
                a.idx_value[base + s_first + lane] = (int64_t)((uint64_t)s_xhi << 32 | s_xlo);
        }
        ns = 0;
    };
    uint32_t pos = 0, nr = 0, miss = 0, skip = 0, kprev = 0;
    int32_t status = LSM_OK;
    for (;;) {
        // ---- exact step at pos (same checks and order as the reference) ----
        // Fields are read straight from the ring; the value length is read
        // speculatively at the previous record's key length, in the same LDS
        // round trip as the key length (keys of one length are the norm).
        const uint32_t rem = n - pos;
        uint32_t klen = 0, vlen = 0, vp = pos;
        uint64_t xval = 0;
        if (rem == 0) break;
        if (rem < 4) {
            status = G == LSM_GRAMMAR_IDX ? LSM_ST_IDX_OVERRUN : LSM_ST_TRUNC_LEN_PREFIX;
            break;
        }
        rd.ensure(rd.h + pos);  // [pos, pos + 1 KiB) landed (and the ring topped up)
        if (G == LSM_GRAMMAR_V) {
            vlen = ufield(pos);
            if (rem - 4 < vlen) { status = LSM_ST_TRUNC_VAL; break; }
        } else if (G == LSM_GRAMMAR_KV) {
            const bool spec_v = kprev <= kChunk - 12 && rem >= 8 + kprev;
            klen = ufield(pos);
            const uint32_t vguess = spec_v ? ufield(pos + 4 + kprev) : 0;
            if (klen > kKeyCap) { status = LSM_ST_KEY_TOO_LONG; break; }
            if (rem - 4 < klen) { status = LSM_ST_TRUNC_KEY; break; }
            vp = pos + 4 + klen;
            const uint32_t rem2 = n - vp;
            if (rem2 < 4) { status = LSM_ST_TRUNC_VLEN; break; }
            if (spec_v && klen == kprev) {
                vlen = vguess;
            } else {
                if (vp + 4 - pos > kChunk) rd.ensure(rd.h + vp);
                vlen = ufield(vp);
            }
            if (vlen > kValCap) { status = LSM_ST_VAL_TOO_LONG; break; }
            if (rem2 - 4 < vlen) { status = LSM_ST_TRUNC_VAL; break; }
            kprev = klen;
        } else {
            klen = ufield(pos);
            if ((uint64_t)rem < 12ull + klen) { status = LSM_ST_IDX_OVERRUN; break; }
            vp = pos + 4 + klen;
            if (vp + 8 - pos > kChunk) rd.ensure(rd.h + vp);
            xval = (uint64_t)ufield(vp + 4) << 32 | ufield(vp);
            vlen = 8;
        }
        if (nr >= cap) { status = LSM_ST_CAPACITY; break; }
        if (ns == 0) s_first = nr;
        if (lane == ns) {
            s_pos = pos;
            s_k = klen;
            s_v = vlen;
            if (G == LSM_GRAMMAR_IDX) {
                s_xlo = (uint32_t)xval;
                s_xhi = (uint32_t)(xval >> 32);
            }
        }
        if (++ns == kWave) flush_stage();
        nr++;
        const uint32_t S = G == LSM_GRAMMAR_V ? 4 + vlen : G == LSM_GRAMMAR_KV ? 8 + klen + vlen
                                                                              : 12 + klen;
        pos += S;

        // ---- speculative runs of records shaped like the last one ----
        // Back off after runs that verified nothing (blocks of varied record
        // shapes, config 5): skip the next 1, 3, 7, 15 attempts.
        if (skip || (a.dbg & 1)) {
            if (skip) skip--;
            continue;
        }
        flush_stage();
        for (bool first = true;; first = false) {
            if (pos >= n) break;
            // wait for the span the run can verify (64 records): all of a block
            // that fits the ring (its chunks were issued together), at most
            // half the ring otherwise, so the younger half stays in flight
            const uint32_t kSpanMax = (rd.nchunks <= NCH ? NCH : NCH / 2) * kChunk;
            const uint64_t span = (uint64_t)S * kWave + 8;
            rd.ensure(rd.h + pos, span < kSpanMax ? (uint32_t)span : kSpanMax);
            uint32_t res = rd.landed * kChunk;  // resident stream end
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
            if (first) {
                if (j == 0) {
                    miss = miss < 4 ? miss + 1 : 4;
                    skip = (1u << miss) - 1;
                } else {
                    miss = 0;
                }
            }
            if (j < 64) break;
        }
    }
    flush_stage();
    if (lane == 0) {
        a.nrec[b] = nr;
        a.status[b] = status;
    }
}

// ---- v2: the chase with the fewest scalar instructions -------------------
//
// The exact step is a serial chain, and a wave-uniform chain runs on the CU's
// one scalar unit, shared by all 32 resident waves: PMC on config 5 (record
// shapes vary, so speculative runs rarely verify) counted 107 SALU
// instructions per record for decode_block_spec, 74% of the kernel time at one
// SALU issue per cycle.  v2 keeps the same semantics with a leaner step:
//  * one compare decides whether the bytes are landed (`lim`), the ring
//    bookkeeping only runs when a step crosses it;
//  * blocks that fit the ring are read without modulo arithmetic (LIN);
//  * the value length is read at the previous key length in the same LDS
//    round trip as the key length;
//  * descriptors are staged branch-free (v_cndmask) and stored 64 at a time;
//  * error statuses are only computed on the (one) failing record.
// Speculative runs are unchanged.
// A wave-uniform value moved into a VGPR, so the arithmetic that depends on
// it stays on the vector ALU (the compiler would otherwise keep a uniform
// chain on the CU's single scalar unit).
__device__ __forceinline__ uint32_t to_vgpr(uint32_t s) {
    uint32_t v;
    __asm__ __volatile__("v_mov_b32 %0, %1" : "=v"(v) : "s"(s));
    return v;
}

// Decode the byte range [off, off + n) of a.in as one block whose records
// go to slots base.. (capacity ncap); returns the record count, the status
// and the position where the chase stopped.  Records that start at or past
// `stop` are not decoded (a clean stop; stop = n decodes the whole range).
template <int G, uint32_t NCH, bool LIN>
__device__ void decode_range_v2(const DecodeArgs &a, uint32_t *ring, uint64_t off, uint32_t n,
                                uint64_t base, uint32_t ncap, uint32_t &nr_out, int32_t &st_out,
                                uint32_t stop, uint32_t &pos_out) {
    constexpr uint32_t kWords = NCH * kChunk / 4;
    const uint32_t lane = lane_id();
    BlockReaderT<NCH> rd;
    rd.init(ring, a.in, off, n);

    // Block bytes below `lim` (and at or above the last anchor) are landed.
    uint32_t lim = 0;
    auto need = [&](uint32_t p, uint32_t len) {
        if ((uint64_t)p + len <= lim) return;
        rd.ensure(rd.h + p, LIN ? rd.total : len);
        lim = rd.landed >= rd.nchunks ? n : rd.landed * kChunk - rd.h;
    };
    auto word = [&](uint32_t w) -> uint32_t { return LIN ? ring[w] : ring[w % kWords]; };
    auto fld = [&](uint32_t p) -> uint32_t {  // wave-uniform u32 at block position p
        const uint32_t sb = rd.h + p;
        const uint32_t w = sb >> 2;
        return uni(funnel(word(w), word(w + 1), sb));
    };
    auto lds_u32 = [&](uint32_t p) -> uint32_t {  // per-lane u32 at block position p
        const uint32_t sb = rd.h + p;
        const uint32_t w = sb >> 2;
        return funnel(word(w), word(w + 1), sb);
    };

    uint32_t s_pos = 0, s_k = 0, s_v = 0, s_xlo = 0, s_xhi = 0, ns = 0, s_first = 0;
    uint32_t pos = 0, nr = 0, kprev = 0xFFFFFFFFu, miss = 0, skip = 0;
    auto flush = [&]() {
        if (ns) {
            if (lane < ns) {
                const uint64_t ro = off + s_pos;
                u32x4 d;
                d.x = (uint32_t)ro;
                d.y = (uint32_t)(ro >> 32);
                d.z = s_k;
                d.w = s_v;
                a.desc[base + s_first + lane] = d;
                if (G == LSM_GRAMMAR_IDX && a.idx_value)
                    a.idx_value[base + s_first + lane] = (int64_t)((uint64_t)s_xhi << 32 | s_xlo);
            }
            ns = 0;
        }
    };
    auto gverify = [&](uint32_t K, uint32_t V, uint32_t S) {
        constexpr uint32_t T = 8;  // 64-record rounds per batch (a 64 KiB block of 124 B records in one)
        const uint32_t cnt = (n - pos) / S;  // candidates wholly inside the block
        uint32_t i0 = 0;
        while (i0 < cnt) {
            uint32_t kw0[T], kw1[T], vw0[T], vw1[T], sb[T];
#pragma unroll
            for (uint32_t t = 0; t < T; t++) {
                const uint32_t i = i0 + t * kWave + lane;
                sb[t] = rd.h + pos + i * S;  // no wrap: i < cnt keeps it inside the block
                const uint32_t sk = (i < cnt ? sb[t] : 0u) & ~3u;
                const uint32_t svv = (i < cnt ? sb[t] + (G == LSM_GRAMMAR_KV ? 4 + K : 0u) : 0u) & ~3u;
                kw0[t] = ld_b32(rd.rsrc, sk);
                kw1[t] = ld_b32(rd.rsrc, sk + 4);
                if (G == LSM_GRAMMAR_KV) {
                    vw0[t] = ld_b32(rd.rsrc, svv);
                    vw1[t] = ld_b32(rd.rsrc, svv + 4);
                }
            }
            uint32_t f = T * kWave;
#pragma unroll
            for (uint32_t t = 0; t < T; t++) {
                const uint32_t i = i0 + t * kWave + lane;
                const uint32_t k = funnel(kw0[t], kw1[t], sb[t]);
                bool ok = i < cnt && nr + i < ncap;
                if (G == LSM_GRAMMAR_KV) {
                    const uint32_t v = funnel(vw0[t], vw1[t], sb[t] + 4 + K);
                    ok = ok && k == K && v == V;
                } else {
                    ok = ok && k == V;
                }
                const uint64_t m = __ballot(ok);
                const uint32_t jt = m == ~0ull ? 64u : (uint32_t)__builtin_ctzll(~m);
                if (f == T * kWave && jt < 64) f = t * kWave + jt;
                if (ok && t * kWave + lane < f) {
                    const uint64_t ro = off + (sb[t] - rd.h);
                    u32x4 d;
                    d.x = (uint32_t)ro;
                    d.y = (uint32_t)(ro >> 32);
                    d.z = K;
                    d.w = V;
                    a.desc[base + nr + i] = d;
                }
            }
            const uint32_t take = f < cnt - i0 ? f : cnt - i0;
            i0 += take;
            if (take < T * kWave) break;
        }
        const uint32_t got = i0 < cnt ? i0 : cnt;
        nr += got;
        pos += got * S;
    };
    int32_t status = LSM_OK;
    for (;;) {
        // ---- exact step at pos (same checks and order as the reference) ----
        const uint32_t rem = n - pos;
        if (rem == 0 || pos >= stop) break;
        if (rem < 4) {
            status = G == LSM_GRAMMAR_IDX ? LSM_ST_IDX_OVERRUN : LSM_ST_TRUNC_LEN_PREFIX;
            break;
        }
        need(pos, rem < kChunk ? rem : kChunk);
        uint32_t K = 0, V, S;
        uint64_t x = 0;
        if (G == LSM_GRAMMAR_V) {
            V = fld(pos);  // data.go:58-76
            if (rem - 4 < V) { status = LSM_ST_TRUNC_VAL; break; }
            S = 4 + V;
        } else if (G == LSM_GRAMMAR_KV) {
            // kv.go:77-115; the guess at kprev lies inside the landed KiB
            const bool sv = kprev <= kChunk - 8;
            K = fld(pos);
            const uint32_t vg = sv ? fld(pos + 4 + kprev) : 0u;
            if (K > kKeyCap) { status = LSM_ST_KEY_TOO_LONG; break; }
            if (rem - 4 < K) { status = LSM_ST_TRUNC_KEY; break; }
            const uint32_t vp = pos + 4 + K;
            const uint32_t rem2 = n - vp;
            if (rem2 < 4) { status = LSM_ST_TRUNC_VLEN; break; }
            if (sv && K == kprev) {
                V = vg;
            } else {
                need(vp, rem2 < kChunk ? rem2 : kChunk);
                V = fld(vp);
            }
            if (V > kValCap) { status = LSM_ST_VAL_TOO_LONG; break; }
            if (rem2 - 4 < V) { status = LSM_ST_TRUNC_VAL; break; }
            kprev = K;
            S = 8 + K + V;
        } else {
            K = fld(pos);  // index.go:70-98
            if ((uint64_t)rem < 12ull + K) { status = LSM_ST_IDX_OVERRUN; break; }
            const uint32_t vp = pos + 4 + K;
            need(vp, 8);
            x = (uint64_t)fld(vp + 4) << 32 | fld(vp);
            V = 8;
            S = 12 + K;
        }
        if (nr >= ncap) { status = LSM_ST_CAPACITY; break; }
        if (ns == 0) s_first = nr;
        {
            const bool me = lane == ns;
            s_pos = me ? pos : s_pos;
            s_k = me ? K : s_k;
            s_v = me ? V : s_v;
            if (G == LSM_GRAMMAR_IDX) {
                s_xlo = me ? (uint32_t)x : s_xlo;
                s_xhi = me ? (uint32_t)(x >> 32) : s_xhi;
            }
        }
        if (++ns == kWave) flush();
        if (nr == 0) stamp(1);
        nr++;
        pos += S;
        if (a.dbg & 4) break;

        // ---- records of varying shape: the VALU chain ----
        // After a failed run (skip > 0) the following records are chased with
        // the cursor in a VGPR: all lanes compute the same step, the checks
        // combine into one ballot and the scalar unit only counts.  The step
        // guesses the previous record's key length and reads the value length
        // there in the same LDS round trip (re-read when the key length
        // differs); any record it cannot vouch for (a key over 1 KiB, bytes
        // not yet landed, an error, the block end, capacity) drops back to the
        // exact step above.
        if (skip) {
            skip--;
            if (G == LSM_GRAMMAR_KV && kprev <= kChunk - 8) {
                uint32_t vpos = to_vgpr(pos), kp = to_vgpr(kprev);
                while (nr < ncap) {
                    const uint32_t sb = rd.h + vpos, sv = sb + 4 + kp;
                    const uint32_t k = funnel(word(sb >> 2), word((sb >> 2) + 1), sb);
                    uint32_t v = funnel(word(sv >> 2), word((sv >> 2) + 1), sv);
                    // a key of another length: the value length is elsewhere
                    // (one more LDS round trip, still on the vector ALU)
                    if (!__ballot(k == kp) && __ballot(k <= kChunk - 8)) {
                        const uint32_t sw = sb + 4 + k;
                        v = funnel(word(sw >> 2), word((sw >> 2) + 1), sw);
                    }
                    const uint32_t rem = n - vpos;
                    const bool ok = (k <= kChunk - 8) & (vpos <= lim) & (lim - vpos >= 8 + k) &
                                    (v <= kValCap) & (rem - 8 - k >= v) & (vpos < stop);
                    if (!__ballot(ok)) break;
                    if (ns == 0) s_first = nr;
                    const bool me = lane == ns;
                    s_pos = me ? vpos : s_pos;
                    s_k = me ? k : s_k;
                    s_v = me ? v : s_v;
                    if (++ns == kWave) flush();
                    nr++;
                    vpos += 8 + k + v;
                    kp = k;
                }
                pos = uni(vpos);
                kprev = uni(kp);
            } else if (G == LSM_GRAMMAR_V) {
                uint32_t vpos = to_vgpr(pos);
                while (nr < ncap) {
                    const uint32_t sb = rd.h + vpos;
                    const uint32_t v = funnel(word(sb >> 2), word((sb >> 2) + 1), sb);
                    const uint32_t rem = n - vpos;
                    const bool ok = (vpos <= lim) & (lim - vpos >= 4u) & (rem - 4 >= v) &
                                    (vpos < stop);
                    if (!__ballot(ok)) break;
                    if (ns == 0) s_first = nr;
                    const bool me = lane == ns;
                    s_pos = me ? vpos : s_pos;
                    s_k = me ? 0u : s_k;
                    s_v = me ? v : s_v;
                    if (++ns == kWave) flush();
                    nr++;
                    vpos += 4 + v;
                }
                pos = uni(vpos);
            }
            continue;
        }
        if (a.dbg & 1) continue;
        flush();
        for (bool first = true;; first = false) {
            if (pos >= n) break;
            // wait for the span the run can verify (64 records): all of a
            // block that fits the ring, half the ring otherwise (the other
            // half stays in flight while the run is checked)
            const uint32_t span_max = (LIN ? NCH : NCH / 2) * kChunk;
            const uint64_t span = (uint64_t)S * kWave + 8;
            const uint32_t want = span < span_max ? (uint32_t)span : span_max;
            need(pos, n - pos < want ? n - pos : want);
            const uint64_t pe = (uint64_t)pos + (uint64_t)(lane + 1) * S;  // record end
            const uint32_t p = pos + lane * S;
            bool ok = pe <= lim && nr + lane < ncap && p < stop;
            uint64_t xx = 0;
            if (ok) {
                if (G == LSM_GRAMMAR_V) {
                    ok = lds_u32(p) == V;
                } else if (G == LSM_GRAMMAR_KV) {
                    ok = (int)(lds_u32(p) == K) & (int)(lds_u32(p + 4 + K) == V);
                } else {
                    ok = lds_u32(p) == K;
                    xx = (uint64_t)lds_u32(p + 8 + K) << 32 | lds_u32(p + 4 + K);
                }
            }
            const uint64_t m = __ballot(ok);
            const uint32_t j = m == ~0ull ? 64u : (uint32_t)__builtin_ctzll(~m);
            if (lane < j) {
                const uint64_t ro = off + p;
                u32x4 d;
                d.x = (uint32_t)ro;
                d.y = (uint32_t)(ro >> 32);
                d.z = K;
                d.w = V;
                a.desc[base + nr + lane] = d;
                if (G == LSM_GRAMMAR_IDX && a.idx_value) a.idx_value[base + nr + lane] = (int64_t)xx;
            }
            // the run ended at the landed limit, not at a mismatch
            const bool at_lim = j == 64 || (uint64_t)pos + (uint64_t)(j + 1) * S > lim;
            nr += j;
            pos += j * S;
            if (first) {
                if (j == 0) {
                    miss = miss < 4 ? miss + 1 : 4;
                    skip = (1u << miss) - 1;
                } else {
                    miss = 0;
                }
            }
            if (!LIN && at_lim && j >= 4 && G != LSM_GRAMMAR_IDX && (a.dbg & 8) && stop >= n) {
                // A full run in a streamed block: test the same hypothesis on
                // the rest of the block straight from global memory, 256
                // records per batch with all their loads in flight (the ring
                // keeps ~2 KiB in flight per wave, too little for 64 KiB
                // blocks at 25 waves per CU).  Verified records are exactly
                // the chase's records (each check reads the record's own
                // fields); the first mismatch goes back to the exact step.
                gverify(K, V, S);
                stamp(2);
                break;
            }
            // a run cut short by the landed limit goes on once more bytes
            // have landed (no exact step in between); a mismatch ends it
            if (j < 64 && !(at_lim && j > 0)) break;
        }
    }
    flush();
    nr_out = nr;
    st_out = status;
    pos_out = pos;
}

template <int G, uint32_t NCH, bool LIN>
__device__ void decode_block_v2(const DecodeArgs &a, uint32_t b, uint32_t *ring, uint64_t off,
                                uint32_t n) {
    uint64_t base, cap;
    record_slots<G>(a, b, off, n, base, cap);
    uint32_t nr, end;
    int32_t st;
    decode_range_v2<G, NCH, LIN>(a, ring, off, n, uni64(base),
                                 uni(cap < 0xFFFFFFFFull ? (uint32_t)cap : 0xFFFFFFFFu), nr, st, n,
                                 end);
    if (lane_id() == 0) {
        a.nrec[b] = nr;
        a.status[b] = st;
    }
}

// Either form of the range decoder: linear when the range fits the ring.
template <int G, uint32_t NCH>
__device__ void decode_range_any(const DecodeArgs &a, uint32_t *ring, uint64_t off, uint32_t n,
                                 uint64_t base, uint32_t ncap, uint32_t &nr, int32_t &st,
                                 uint32_t stop = 0xFFFFFFFFu, uint32_t *end = nullptr) {
    uint32_t e;
    if (((off & 15) + (uint64_t)n + 15) / 16 * 16 <= NCH * kChunk)
        decode_range_v2<G, NCH, true>(a, ring, off, n, base, ncap, nr, st, stop, e);
    else
        decode_range_v2<G, NCH, false>(a, ring, off, n, base, ncap, nr, st, stop, e);
    if (end) *end = e;
}

// One wave (and one workgroup) per block; NCH x 1 KiB ring plus a guard
// dword so linear reads of a block's last field stay inside the array.
template <int G, uint32_t NCH>
__global__ __launch_bounds__(64) void decode_v2_kernel(DecodeArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t ring[NCH * kChunk / 4 + 4];
    const uint32_t b = blockIdx.x;
    stamp(0);
    const uint64_t off = uni64(a.blk_off[b]);
    const uint32_t n = uni(a.blk_len[b]);
    if (a.split && (off & 15) + (uint64_t)n > NCH * kChunk) return;
    if (((off & 15) + (uint64_t)n + 15) / 16 * 16 <= NCH * kChunk)
        decode_block_v2<G, NCH, true>(a, b, ring, off, n);
    else
        decode_block_v2<G, NCH, false>(a, b, ring, off, n);
    stamp(3);
}

template <int G, uint32_t NCH>
int launch_v2(const DecodeArgs &a, hipStream_t s) {
    hipLaunchKernelGGL((decode_v2_kernel<G, NCH>), dim3(a.nblk), dim3(kWave), 0, s, a);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
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
        if (a.split && (off & 15) + (uint64_t)n > kRingBytes) continue;
        decode_block_spec<G>(a, b, ring[wave], off, n);
    }
    stamp(3);
}

// ---- blocks larger than the 4 KiB ring ------------------------------------
//
// A 4 KiB ring keeps at most 3 KiB in flight per wave, which streams a 64 KiB
// block at a fraction of the HBM rate (decode64k 0.56 of peak, config 5
// 0.35).  Blocks with h + n > 4 KiB are therefore left by the small-block
// kernel (a.split) to this persistent one: W one-wave workgroups, each with a
// 16 KiB ring (up to 15 KiB in flight, 10 waves per CU by LDS), walk the
// block list with stride W.  Lane l of wave w looks at block r0 + l*W and a
// ballot picks the large ones, so a batch without large blocks costs one
// metadata load per wave.
constexpr uint32_t kLargeNCH = 16;

template <int G, uint32_t NCH>
__global__ __launch_bounds__(64) void decode_large_kernel(DecodeArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t ring[NCH * kChunk / 4 + 4];
    const uint64_t W = gridDim.x;
    const uint32_t lane = lane_id();
    for (uint64_t r0 = blockIdx.x; r0 < a.nblk; r0 += W * kWave) {
        const uint64_t b = r0 + lane * W;
        uint64_t off = 0;
        uint32_t n = 0;
        bool big = false;
        if (b < a.nblk) {
            off = a.blk_off[b];
            n = a.blk_len[b];
            big = (off & 15) + (uint64_t)n > kRingBytes;
        }
        uint64_t m = __ballot(big);
        while (m) {
            const uint32_t l = uni((uint32_t)__builtin_ctzll(m));
            m &= m - 1;
            const uint64_t offj = uni64((uint32_t)__builtin_amdgcn_readlane((uint32_t)off, l) |
                                        (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(off >> 32), l) << 32);
            const uint32_t nj = uni(__builtin_amdgcn_readlane(n, l));
            decode_block_v2<G, NCH, false>(a, (uint32_t)(r0 + (uint64_t)l * W), ring, offj, nj);
        }
    }
}

template <int G, uint32_t NCH>
int launch_large(lsm_ctx *ctx, const DecodeArgs &a, hipStream_t s) {
    // resident one-wave workgroups per CU: the 160 KiB LDS over the ring
    constexpr uint32_t per_cu = 160 / NCH;
    const uint32_t cus = ctx ? (uint32_t)lsm_ctx_num_cus(ctx) : 256u;
    uint64_t grid = (uint64_t)cus * per_cu;
    if (grid > a.nblk) grid = a.nblk;
    if (grid == 0) return 0;
    hipLaunchKernelGGL((decode_large_kernel<G, NCH>), dim3((uint32_t)grid), dim3(kWave), 0, s, a);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
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
            if (!strcmp(e, "large8")) return 40;
            if (!strcmp(e, "v2split")) return 41;
            if (!strcmp(e, "v2r4")) return 42;
            if (!strcmp(e, "v2r6")) return 43;
            if (!strcmp(e, "v2r5")) return 44;
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
        // one wave per block, 8 KiB ring: decode4k equal to a 4 KiB ring,
        // decode64k 0.71 vs 0.58 of HBM peak (more in flight per wave)
        case 0: return launch_v2<G, 8>(a, s);
        case 41: {
            // v2 for blocks that fit the 4 KiB ring, then the deep-ring
            // persistent kernel for the larger ones
            DecodeArgs b = a;
            b.split = 1;
            const int rc = launch_v2<G, kNChunk>(b, s);
            return rc ? rc : launch_large<G, kLargeNCH>(ctx, b, s);
        }
        case 42: return launch_v2<G, kNChunk>(a, s);
        case 43: return launch_v2<G, 6>(a, s);
        case 44: return launch_v2<G, 5>(a, s);
        case 40: {
            DecodeArgs b = a;
            b.split = 1;
            const int rc = launch_spec<G, 1, 1>(b, s);
            return rc ? rc : launch_large<G, 8>(ctx, b, s);
        }
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

// ---- whole .sst files: SSTable.DecodeFrom + DecodeDataBlock + join ---------
//
// SURVEY.md §8(f) row f1.  go-lsm decodes a file's index region and data
// region by two serial chases (index.go:61-101, data.go:49-79) and joins
// value i with index key i (sstable.go:248-268).  Here, per file:
//   1. sst_index_kernel: every workgroup parses the framing (header, filter
//      prefix, footer; sstable.go:87-128); then all threads test the stride
//      hypothesis "every index entry has the first entry's key length" on
//      the whole index region at once.  Entry i verified <=> its key length
//      field holds K0, so the serial chase visits exactly these entries.
//   2. sst_index_fixup_kernel: one wave chases the index from the first
//      entry the hypothesis failed on (decode_range_v2, exact semantics).
//   3. sst_data_verify_kernel: the values are located by the index offsets
//      (SSTable.EncodeTo writes value i at Indexes[i].Offset,
//      sstable.go:164-169); value i is verified when it starts where value
//      i-1 ended (value 0 at DataHandle.Offset) and ends where value i+1
//      starts (the last one at the end of the region).  The verified values
//      are exactly the serial chase's.
//   4. sst_data_fixup_kernel: one wave chases the data region from the first
//      unverified value, then applies GetKeyValuePairs' count rules and
//      writes the per-file lsm_sst_meta.
// A well-formed file costs two parallel passes; a corrupted one falls back
// to the exact chase only from the first entry that cannot be vouched for.

// Range-checked little-endian reads at byte offsets of one file image.
struct ImgReader {
    rsrc_t r;
    uint32_t h;  // image start inside its 4-byte aligned base
    __device__ void init(const uint8_t *img, uint64_t foff, uint64_t n) {
        const uint64_t a0 = foff & ~(uint64_t)3;
        h = (uint32_t)(foff - a0);
        uint64_t tot = (h + n + 7) & ~(uint64_t)3;
        if (tot > 0xFFFFFFF0ull) tot = 0xFFFFFFF0ull;
        r = make_rsrc(img + a0, (uint32_t)tot);
    }
    __device__ uint32_t u32(uint64_t p) const {
        const uint32_t s = h + (uint32_t)p;
        return funnel(ld_b32(r, s & ~3u), ld_b32(r, (s & ~3u) + 4), s);
    }
    __device__ uint64_t u64(uint64_t p) const { return (uint64_t)u32(p + 4) << 32 | u32(p); }
    __device__ uint64_t u64be(uint64_t p) const { return __builtin_bswap64(u64(p)); }
};

struct SstWork {
    lsm_sst_meta m;
    uint64_t io, il, dof, dl;  // index / data regions to decode (image-relative)
    uint64_t base, cap;        // record slots of the file
    uint32_t k0, spec_cnt;     // index stride hypothesis: key length, entries to test
    uint32_t idx_overrun;      // IndexHandle.Size runs past the end of the file
    uint32_t data_neg;         // DataHandle.Offset < 0: the seek fails
};

// SSTable.DecodeFrom's framing (sstable.go:87-128) as the oracle restates it
// (oracle/lsm_oracle.c ora_sst_decode); one thread.
__device__ void sst_parse(const ImgReader &R, uint64_t n, SstWork &w) {
    lsm_sst_meta &m = w.m;
    uint64_t pos = 0;
    for (int j = 0; j < 2; j++) {  // Header.DecodeFrom header.go:40-52 (Key: no cap)
        if (n - pos < 4) { m.stage = LSM_SST_HEADER; return; }
        const uint32_t kl = R.u32(pos);
        if (n - pos - 4 < kl) { m.stage = LSM_SST_HEADER; return; }
        if (j == 0) { m.min_key_off = pos + 4; m.min_key_len = kl; }
        else { m.max_key_off = pos + 4; m.max_key_len = kl; }
        pos += 4 + (uint64_t)kl;
    }
    // Filter.DecodeFrom bloom.go:453-469 -> ReadFrom :262-281 -> bitset ReadFrom
    if (n - pos < 8) { m.stage = LSM_SST_FILTER; return; }
    const uint64_t L = R.u64(pos);
    if (L > n - pos - 8 || L < 24) { m.stage = LSM_SST_FILTER; return; }
    const uint64_t fm = R.u64be(pos + 8), fk = R.u64be(pos + 16), nb = R.u64be(pos + 24);
    if ((nb + 63) / 64 > (L - 24) / 8) { m.stage = LSM_SST_FILTER; return; }
    m.filter_m = fm;
    m.filter_k = fk;
    m.filter_nbits = nb;
    m.filter_words_off = pos + 32;
    // DecodeFooterFrom sstable.go:195-212
    if (n < 32) { m.stage = LSM_SST_FOOTER; return; }
    m.data_off = (int64_t)R.u64(n - 32);
    m.data_size = (int64_t)R.u64(n - 24);
    m.idx_off = (int64_t)R.u64(n - 16);
    m.idx_size = (int64_t)R.u64(n - 8);
    // seek to IndexHandle.Offset; IndexBlock.DecodeFrom rejects a negative size
    if (m.idx_off < 0 || m.idx_size < 0) { m.stage = LSM_SST_INDEX; return; }
    const uint64_t io = (uint64_t)m.idx_off, avail = io <= n ? n - io : 0;
    w.io = io;
    w.il = (uint64_t)m.idx_size < avail ? (uint64_t)m.idx_size : avail;
    w.idx_overrun = (uint64_t)m.idx_size > avail;  // the file ends before the limit
    // DecodeDataBlock: DataBlock.DecodeFrom(file, DataHandle.Size), size <= 0 = to EOF
    w.data_neg = m.data_off < 0;
    const uint64_t dof = w.data_neg ? 0 : (uint64_t)m.data_off;
    const uint64_t davail = dof <= n ? n - dof : 0;
    w.dof = dof;
    w.dl = (m.data_size > 0 && (uint64_t)m.data_size < davail) ? (uint64_t)m.data_size : davail;
}

struct SstArgs {
    const uint8_t *img;
    const uint64_t *file_off, *file_len;
    uint32_t nfile;
    const uint64_t *rec_base;
    lsm_sst_meta *meta;
    u32x4 *idx_desc;
    int64_t *idx_value;
    u32x4 *data_desc;
    SstWork *work;
    uint32_t *fail;  // [2f] first unverified index entry, [2f+1] first unverified value
};

__device__ __forceinline__ void sst_slots(const SstArgs &a, uint32_t f, uint64_t foff, uint64_t n,
                                          uint64_t &base, uint64_t &cap) {
    if (a.rec_base) {
        base = a.rec_base[f];
        cap = a.rec_base[f + 1] - base;
    } else {
        base = foff / 4;
        cap = (foff + n) / 4 - base;
    }
}

__global__ __launch_bounds__(256) void sst_index_kernel(SstArgs a) {
    __shared__ SstWork W;
    const uint32_t f = blockIdx.y;
    const uint64_t foff = a.file_off[f], n = a.file_len[f];
    ImgReader R;
    R.init(a.img, foff, n);
    if (threadIdx.x == 0) {
        memset(&W, 0, sizeof(W));
        sst_parse(R, n, W);
        sst_slots(a, f, foff, n, W.base, W.cap);
        if (W.m.stage == 0 && W.il >= 4) {
            W.k0 = R.u32(W.io);
            const uint64_t cnt = W.il / (12ull + W.k0);
            const uint64_t lim = W.cap < 0xFFFFFFFFull ? W.cap : 0xFFFFFFFFull;
            W.spec_cnt = (uint32_t)(cnt < lim ? cnt : lim);
        }
        if (blockIdx.x == 0) a.work[f] = W;
    }
    __syncthreads();
    if (W.m.stage != 0) return;
    const uint64_t S = 12ull + W.k0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < W.spec_cnt;
         i += gridDim.x * blockDim.x) {
        const uint64_t p = W.io + (uint64_t)i * S;
        if (R.u32(p) == W.k0) {
            const uint64_t ro = foff + p;
            u32x4 d;
            d.x = (uint32_t)ro;
            d.y = (uint32_t)(ro >> 32);
            d.z = W.k0;
            d.w = 8;
            a.idx_desc[W.base + i] = d;
            a.idx_value[W.base + i] = (int64_t)R.u64(p + 4 + W.k0);
        } else {
            atomicMin(&a.fail[2 * f], i);
        }
    }
}

__global__ __launch_bounds__(64) void sst_index_fixup_kernel(SstArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t ring[8 * kChunk / 4 + 4];
    const uint32_t f = blockIdx.x;
    SstWork &W = a.work[f];
    if (uni((uint32_t)W.m.stage) != 0) return;
    const uint32_t spec = uni(W.spec_cnt);
    const uint32_t fl = uni(a.fail[2 * f]);
    const uint32_t i0 = fl < spec ? fl : spec;
    const uint64_t S = 12ull + uni(W.k0), il = uni64(W.il);
    const bool overrun = uni(W.idx_overrun) != 0;
    uint32_t nidx;
    int32_t st = LSM_OK;
    if (i0 == spec && (uint64_t)spec * S == il && !overrun) {
        nidx = spec;
    } else {
        DecodeArgs d = {};
        d.in = a.img;
        d.desc = a.idx_desc;
        d.idx_value = a.idx_value;
        const uint64_t start = (uint64_t)i0 * S, cap = uni64(W.cap);
        uint32_t nr = 0;
        decode_range_any<LSM_GRAMMAR_IDX, 8>(
            d, ring, uni64(a.file_off[f]) + uni64(W.io) + start, (uint32_t)(il - start),
            uni64(W.base) + i0, (uint32_t)(cap - i0 < 0xFFFFFFFFull ? cap - i0 : 0xFFFFFFFFull), nr, st);
        nidx = i0 + nr;
        if (overrun && st == LSM_OK) st = LSM_ST_IDX_OVERRUN;  // index.go:73-91 reads past EOF
    }
    if (lane_id() == 0) {
        W.m.nidx = nidx;
        if (st != LSM_OK) {
            W.m.stage = LSM_SST_INDEX;
            W.m.status = st;
        }
    }
}

__global__ __launch_bounds__(256) void sst_data_verify_kernel(SstArgs a) {
    __shared__ SstWork W;
    const uint32_t f = blockIdx.y;
    if (threadIdx.x == 0) W = a.work[f];
    __syncthreads();
    if (W.m.stage != 0 || W.data_neg) return;
    const uint64_t foff = a.file_off[f];
    ImgReader R;
    R.init(a.img, foff, a.file_len[f]);
    const uint64_t doff = (uint64_t)W.m.data_off, dl = W.dl;
    const uint32_t nidx = W.m.nidx;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nidx;
         i += gridDim.x * blockDim.x) {
        const uint64_t pos = (uint64_t)a.idx_value[W.base + i] - doff;  // value i, region-relative
        bool bad = dl < 4 || pos > dl - 4 || (i == 0 && pos != 0);
        if (!bad) {
            const uint32_t v = R.u32(W.dof + pos);
            const uint64_t e = pos + 4 + v;  // where value i ends
            const uint64_t next = i + 1 < nidx ? (uint64_t)a.idx_value[W.base + i + 1] - doff : dl;
            bad = e > dl || e != next;
            const uint64_t ro = foff + W.dof + pos;
            u32x4 d;
            d.x = (uint32_t)ro;
            d.y = (uint32_t)(ro >> 32);
            d.z = 0;
            d.w = v;
            a.data_desc[W.base + i] = d;
        }
        if (bad) atomicMin(&a.fail[2 * f + 1], i);
    }
}

__global__ __launch_bounds__(64) void sst_data_fixup_kernel(SstArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t ring[8 * kChunk / 4 + 4];
    const uint32_t f = blockIdx.x;
    SstWork &W = a.work[f];
    int32_t stage = (int32_t)uni((uint32_t)W.m.stage);
    int32_t status = (int32_t)uni((uint32_t)W.m.status);
    const uint32_t nidx = uni(W.m.nidx);
    uint32_t ndata = 0;
    if (stage == LSM_SST_OK) {
        if (uni(W.data_neg)) {
            stage = LSM_SST_DATA;  // seek to a negative offset
        } else {
            const uint32_t fl = uni(a.fail[2 * f + 1]);
            const uint32_t f0 = nidx == 0 ? 0u : (fl < nidx ? fl : nidx);
            int32_t st = LSM_OK;
            if (nidx > 0 && f0 == nidx) {
                ndata = nidx;
            } else {
                const uint64_t doff = uni64((uint64_t)W.m.data_off), dl = uni64(W.dl);
                const uint64_t start =
                    f0 == 0 ? 0 : uni64((uint64_t)a.idx_value[uni64(W.base) + f0] - doff);
                DecodeArgs d = {};
                d.in = a.img;
                d.desc = a.data_desc;
                const uint64_t cap = uni64(W.cap);
                uint32_t nr = 0;
                decode_range_any<LSM_GRAMMAR_V, 8>(
                    d, ring, uni64(a.file_off[f]) + uni64(W.dof) + start, (uint32_t)(dl - start),
                    uni64(W.base) + f0,
                    (uint32_t)(cap - f0 < 0xFFFFFFFFull ? cap - f0 : 0xFFFFFFFFull), nr, st);
                ndata = f0 + nr;
            }
            if (st != LSM_OK) {
                stage = LSM_SST_DATA;
                status = st;
            } else if (nidx && ndata && nidx != ndata) {
                stage = LSM_SST_MISMATCH;  // GetKeyValuePairs sstable.go:254-257
            }
        }
    }
    if (lane_id() == 0) {
        lsm_sst_meta m = W.m;
        m.stage = stage;
        m.status = status;
        m.ndata = ndata;
        a.meta[f] = m;
    }
}

// ---- WAL replay: one long KV stream per log ----------
//
// wal.Recover chases a whole log (~1.7 MB, ~44k records for a 2 MiB
// memtable) as one serial chain; one wave per log would take milliseconds.
// The log is cut into 16 KiB segments, one wave each:
//   wal_seg_kernel: two waves per segment guess where its first record starts
//     (the first position from which three records in a row have plausible
//     lengths).  A record is two length-prefixed fields, so a chain started
//     at a value-length field looks just as plausible, one field out of
//     phase, and never meets the true chain: wave 0 chases from the guess g,
//     wave 1 from g + 4 + u32(g) (the record after the value if g was a
//     value length).  Each chases to the first record starting in the next
//     segment and writes its records to a scratch area of its own.
//   wal_stitch_kernel: one wave per log walks the segments in order with the
//     true chain position e (0 at the start).  A chain of the segment that
//     starts at e is the serial chase's (same start, same deterministic
//     chain); if neither does, the segment is chased again from e.  The
//     first error ends the log, as it ends Recover.
//   wal_compact_kernel: each segment's records move to their final slots.
// The result equals one serial chase for any input; guesses only decide how
// much is chased twice.
#ifndef LSM_WAL_SEG_KIB
#define LSM_WAL_SEG_KIB 16  // other sizes: diagnostic builds only (an open parity item)
#endif
constexpr uint32_t kWalSeg = LSM_WAL_SEG_KIB * 1024;
constexpr uint32_t kWalSegSlots = kWalSeg / 8 + 1;  // records starting in a segment

struct WalSeg {
    uint32_t entry, exit, nrec;
    int32_t status;
};

struct WalArgs {
    const uint8_t *wal;
    const uint64_t *wal_off;
    const uint32_t *wal_len;
    uint32_t nwal, segs, max_len;
    lsm_decode_out out;
    WalSeg *seg;      // nwal * segs * 2 (two phases)
    uint32_t *fin;    // nwal * segs * 2: prefix, count | phase << 31
    u32x4 *scratch;   // nwal * segs * 2 * kWalSegSlots
};

__device__ __forceinline__ void wal_slots(const WalArgs &a, uint32_t w, uint64_t &base,
                                          uint64_t &cap) {
    if (a.out.rec_base) {
        base = a.out.rec_base[w];
        cap = a.out.rec_base[w + 1] - base;
    } else {
        const uint64_t o = a.wal_off[w];
        base = o / 8;
        cap = (o + a.wal_len[w]) / 8 - base;
    }
}

__global__ __launch_bounds__(64) void wal_seg_kernel(WalArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t ring[8 * kChunk / 4 + 4];
    const uint32_t s = blockIdx.x >> 1, ph = blockIdx.x & 1, w = blockIdx.y, lane = lane_id();
    const uint32_t len = uni(a.wal_len[w]);
    const uint64_t off = uni64(a.wal_off[w]);
    const uint64_t q = ((uint64_t)w * a.segs + s) * 2 + ph;
    WalSeg &T = a.seg[q];
    const uint32_t start = s * kWalSeg;
    if (start >= len || len > a.max_len) {
        if (lane == 0) T = WalSeg{0xFFFFFFFFu, 0xFFFFFFFFu, 0, 0};
        return;
    }
    uint32_t g = start;
    if (s > 0) {
        // stage up to 4 KiB of the segment head, then test 64 candidate
        // starts per round: records of plausible lengths in a row (key <=
        // 1 KiB, value <= 1 MiB, inside the log), at least two of them read
        // within the staged bytes or one that ends the log; a guess only
        // decides what the stitch must re-chase, never the result
        const uint64_t a0 = (off + start) & ~(uint64_t)15;
        const uint32_t h = (uint32_t)(off + start - a0);
        const uint32_t W = len - start < kRingBytes - 16 ? len - start : kRingBytes - 16;
        const rsrc_t r = make_rsrc(a.wal + a0, (h + W + 15) & ~15u);
#pragma unroll
        for (uint32_t c = 0; c < kNChunk; c++)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                r, (__attribute__((address_space(3))) void *)&ring[c * (kChunk / 4)], 16,
                c * kChunk + lane * 16, 0, 0, kBlockLoadAux);
        __asm__ __volatile__("s_waitcnt vmcnt(0)" ::: "memory");
        auto rd = [&](uint32_t q) -> uint32_t {
            const uint32_t sb = h + q;
            return funnel(ring[sb >> 2], ring[(sb >> 2) + 1], sb);
        };
        const uint32_t rlen = W < 2048 ? W : 2048;
        g = 0xFFFFFFFFu;
        for (uint32_t t0 = 0; t0 < rlen && g == 0xFFFFFFFFu; t0 += kWave) {
            const uint32_t p = t0 + lane;
            bool ok = p < rlen;
            uint32_t q = p, seen = 0;
            for (int rec = 0; rec < 3 && ok; rec++) {
                if ((uint64_t)start + q == len) { seen = 2; break; }  // ends the log exactly
                if (q + 8 > W) break;
                const uint32_t k = rd(q);
                if (k > 1024 || (uint64_t)start + q + 8 + k > len) { ok = false; break; }
                if (q + 8 + k > W) break;
                const uint32_t v = rd(q + 4 + k);
                if (v > (1u << 20) || (uint64_t)start + q + 8 + k + v > len) { ok = false; break; }
                q += 8 + k + v;
                seen++;
            }
            ok = ok && seen >= 2;
            const uint64_t m = __ballot(ok);
            if (m) g = start + t0 + (uint32_t)__builtin_ctzll(m);
        }
        if (g == 0xFFFFFFFFu) g = start;
        if (ph == 1) {  // the other phase: g read as a value length
            const uint32_t v = g - start + 4 <= W ? rd(g - start) : 0xFFFFFFFFu;
            g = (uint64_t)g + 4 + v <= len ? g + 4 + v : len;
        }
    } else if (ph == 1) {
        if (lane == 0) T = WalSeg{0xFFFFFFFFu, 0xFFFFFFFFu, 0, 0};  // segment 0 starts at 0
        return;
    }
    g = uni(g);
    if (g >= len || g >= start + kWalSeg) {
        if (lane == 0) T = WalSeg{g, g, 0, 0};
        return;
    }
    const uint32_t stop = (start + kWalSeg < len ? start + kWalSeg : len) - g;
    DecodeArgs d = {};
    d.in = a.wal;
    d.desc = a.scratch;
    uint32_t nr = 0, endp = 0;
    int32_t st = LSM_OK;
    decode_range_any<LSM_GRAMMAR_KV, 8>(d, ring, off + g, len - g, q * kWalSegSlots, kWalSegSlots,
                                        nr, st, stop, &endp);
    if (lane == 0) T = WalSeg{g, g + endp, nr, st};
}

// Lane-parallel form of wal_seg_kernel (the default).  WAL records are small
// (~40 B for go-lsm's benchmark) and vary in shape, so one wave chasing a
// 16 KiB segment spends its time in ~400 serial exact steps.  Here the
// segment [g, E) (g the segment's guess as above, E its end) is split into
// 64 shares, one per lane:
//   1. lane 0 starts at g; lane l > 0 guesses its first record start (the
//      first position of its share from which two plausible records follow)
//      and chases both field phases (the guess, and the guess read as a value
//      length), each to the first record starting past its share;
//   2. the wave stitches the shares in order from g: the chain that starts
//      where the previous share ended is the serial chase's; if neither
//      does, that share is chased again from the true position;
//   3. each lane writes the descriptors of its accepted chain.
// The result is the serial chase of [g, E) for any input (exact check order
// of kv.go:77-115); the segment is read from an LDS copy (plus 4 KiB past
// its end) and past that through a range-checked buffer resource.
// LDS copy of a segment plus a tail for the chains that cross its end.  The
// copy sets the occupancy (160 KiB LDS per CU): + 1 KiB admits 9 waves per CU
// and measured 603 GiB/s on the wal bench; + 3.5 KiB (8 waves) 552 and + 4 KiB
// (20,496 B: 7 waves) 542.  Reads past the tail go through the buffer resource.
constexpr uint32_t kWalStage = kWalSeg + 1024;
#ifndef LSM_WAL_DBG
#define LSM_WAL_DBG 0  // timing diagnostics only: 1 skips the write-out, 2 phase 1
#endif
constexpr uint32_t kWalStage4k = kWalSeg + 4096;  // LSM_WAL_KERNEL=stage4k (A/B)

struct WalLog {
    rsrc_t r;       // the log's bytes, offsets relative to the aligned base
    uint32_t h;     // log start inside the base
    uint32_t len;
    uint32_t s0;    // LDS copy covers resource offsets [s0, s0 + sz)
    uint32_t sz;
    const uint32_t *lds;
    __device__ __forceinline__ uint32_t rd32(uint32_t x) const {  // bytes [x, x+4) of the log
        const uint32_t o = h + x;
        if (o >= s0 && o + 8 <= s0 + sz) {
            const uint32_t q = o - s0;
            return funnel(lds[q >> 2], lds[(q >> 2) + 1], q);
        }
        const uint32_t oa = o & ~3u;
        return funnel(ld_b32(r, oa), ld_b32(r, oa + 4), o);
    }
    // exact KV record at p < len (kv.go:77-115 / ora_decode_block order)
    __device__ __forceinline__ int32_t record(uint32_t p, uint32_t &kl, uint32_t &vl) const {
        const uint32_t rem = len - p;
        if (rem < 4) return LSM_ST_TRUNC_LEN_PREFIX;
        kl = rd32(p);
        if (kl > kKeyCap) return LSM_ST_KEY_TOO_LONG;
        if (rem - 4 < kl) return LSM_ST_TRUNC_KEY;
        const uint32_t rem2 = rem - 4 - kl;
        if (rem2 < 4) return LSM_ST_TRUNC_VLEN;
        vl = rd32(p + 4 + kl);
        if (vl > kValCap) return LSM_ST_VAL_TOO_LONG;
        if (rem2 - 4 < vl) return LSM_ST_TRUNC_VAL;
        return LSM_OK;
    }
    // chase from p while records start before `end`: count, stop position, status
    __device__ __forceinline__ void chase(uint32_t p, uint32_t end, uint32_t &cnt, uint32_t &exitp,
                                          int32_t &st) const {
        cnt = 0;
        st = LSM_OK;
        while (p < end && p < len) {
            uint32_t kl = 0, vl = 0;
            st = record(p, kl, vl);
            if (st != LSM_OK) break;
            cnt++;
            p += 8 + kl + vl;
        }
        exitp = p;
    }
    // plausible record start (as the segment guess: two records or the log's end)
    __device__ __forceinline__ bool plausible(uint32_t q) const {
        uint32_t seen = 0;
        for (int rec = 0; rec < 2; rec++) {
            if (q == len) return seen >= 1;
            if ((uint64_t)q + 8 > len) return false;
            const uint32_t k = rd32(q);
            if (k > 1024 || (uint64_t)q + 8 + k > len) return false;
            const uint32_t v = rd32(q + 4 + k);
            if (v > (1u << 20) || (uint64_t)q + 8 + k + v > len) return false;
            q += 8 + k + v;
            seen++;
        }
        return true;
    }
};

// One wave serves both phases of a segment: the shares' chains do not depend
// on the segment's entry, only lane 0's does, so they are chased once and
// stitched twice (from g and from g read as a value length).
template <uint32_t STAGE>  // bytes copied to LDS (0: read through the caches)
__global__ __launch_bounds__(64) void wal_seg_lanes_kernel(WalArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t stage[STAGE ? STAGE / 4 + 4 : 4];
    const uint32_t s = blockIdx.x, w = blockIdx.y, lane = lane_id();
    const uint32_t len = uni(a.wal_len[w]);
    const uint64_t off = uni64(a.wal_off[w]);
    const uint64_t q0 = ((uint64_t)w * a.segs + s) * 2;
    const uint32_t start = s * kWalSeg;
    if (start >= len || len > a.max_len) {
        if (lane == 0) a.seg[q0] = a.seg[q0 + 1] = WalSeg{0xFFFFFFFFu, 0xFFFFFFFFu, 0, 0};
        return;
    }
    WalLog L;
    const uint64_t base = off & ~(uint64_t)15;
    L.h = (uint32_t)(off - base);
    L.len = len;
    L.r = make_rsrc(a.wal + base, (L.h + len + 15) & ~15u);
    L.s0 = STAGE ? (L.h + start) & ~15u : 0xFFFFFFF0u;
    L.sz = STAGE;
    L.lds = stage;
    if (STAGE) {
        // the segment + a tail (the loads are already all in flight: staging
        // by buffer_load ... lds measured no faster)
        for (uint32_t c = 0; c < STAGE / 16; c += kWave) {
            const uint32_t o = L.s0 + 16 * (c + lane);
            if (c + lane < STAGE / 16)
                *reinterpret_cast<u32x4 *>(&stage[4 * (c + lane)]) = ld_b128(L.r, o);
        }
        __syncthreads();
    }
    uint32_t g = start, g1 = 0xFFFFFFFFu;  // entries of phase 0 and phase 1
    if (s > 0) {  // the segment's guess: the first plausible start in its first 2 KiB
        g = 0xFFFFFFFFu;
        const uint32_t span = len - start < 2048 ? len - start : 2048;
        for (uint32_t t0 = 0; t0 < span && g == 0xFFFFFFFFu; t0 += kWave) {
            const uint32_t p = start + t0 + lane;
            const uint64_t m = __ballot(t0 + lane < span && L.plausible(p));
            if (m) g = start + t0 + (uint32_t)__builtin_ctzll(m);
        }
        if (g == 0xFFFFFFFFu) g = start;
        g = uni(g);
        const uint32_t v = (uint64_t)g + 4 <= len ? L.rd32(g) : 0xFFFFFFFFu;
        g1 = uni((uint64_t)g + 4 + v <= len ? g + 4 + v : len);
    }
    const uint32_t E = start + kWalSeg < len ? start + kWalSeg : len;
    // 1. shares of [start, E): lane 0's chains are the two entries themselves.
    //    A share width of a multiple of 128 B would start every lane on the
    //    same LDS bank; widths of 4 mod 8 dwords spread them.
    uint32_t W = (E - start + kWave - 1) / kWave;
    W = (W + 3) & ~3u;
    if ((W / 4) % 8 != 4) W += 4 * ((12 - (W / 4) % 8) % 8);
    const uint32_t ss = start + lane * W < E ? start + lane * W : E;
    const uint32_t se = ss + W < E ? ss + W : E;
    uint32_t e0 = 0xFFFFFFFFu, e1 = 0xFFFFFFFFu, c0 = 0, c1 = 0, x0 = 0, x1 = 0;
    int32_t st0 = LSM_OK, st1 = LSM_OK;
    if (lane > 0 && ss < se) {
        for (uint32_t p = ss; p < se; p++)
            if (L.plausible(p)) { e0 = p; break; }
        if (e0 != 0xFFFFFFFFu && (uint64_t)e0 + 4 <= len) {
            const uint32_t v = L.rd32(e0);
            if ((uint64_t)e0 + 4 + v <= len) e1 = e0 + 4 + v;
        }
    }
    // A guess at or past the share's end is a chain with no records that
    // passes its position through (exit = the guess); chase() returns exactly
    // that.  Leaving its exit unset once made a share holding only a value
    // field report exit 0 when the previous chain ended on that guess.
    if (e0 != 0xFFFFFFFFu) L.chase(e0, se, c0, x0, st0);
    if (e1 != 0xFFFFFFFFu) L.chase(e1, se, c1, x1, st1);
    // 2. + 3. per phase: stitch from the entry, then write the accepted chains
    for (uint32_t ph = 0; ph < ((LSM_WAL_DBG & 2) ? 1 : 2); ph++) {
        const uint64_t q = q0 + ph;
        const uint32_t gp = ph ? g1 : g;
        if (ph == 1 && s == 0) {  // segment 0 starts at 0
            if (lane == 0) a.seg[q] = WalSeg{0xFFFFFFFFu, 0xFFFFFFFFu, 0, 0};
            break;
        }
        if (gp >= E) {
            if (lane == 0) a.seg[q] = WalSeg{gp, gp, 0, 0};
            continue;
        }
        uint32_t e = gp, acc_entry = 0xFFFFFFFFu, acc_cnt = 0, total = 0;
        int32_t status = LSM_OK;
        bool dead = false;
        // fast stitch: the share k holding the entry is chased exactly; after
        // it, lane l's choice of chain (0: from e0, 1: from e1) is a function
        // of lane l-1's choice (its chain's exit matched against lane l's
        // entries); a 6-step scan composes these maps across the lanes.  Any
        // miss (a wrong guess, or a record longer than a share) falls back to
        // the serial stitch below.
        bool fast = false;
        {
            const uint32_t k = (gp - start) / W;
            const uint32_t last = (E - 1 - start) / W < kWave - 1 ? (E - 1 - start) / W : kWave - 1;
            const uint32_t sek = uni(__builtin_amdgcn_readlane(se, k));
            uint32_t ck, xk;
            int32_t stk;
            L.chase(gp, sek, ck, xk, stk);
            ck = uni(ck);
            xk = uni(xk);
            stk = (int32_t)uni((uint32_t)stk);
            auto match = [&](uint32_t x) -> uint32_t {
                return (e0 != 0xFFFFFFFFu && x == e0) ? 0u : (e1 != 0xFFFFFFFFu && x == e1) ? 1u : 2u;
            };
            // map from lane l-1's choice to lane l's, as h0 | h1 << 4 (2 = miss)
            const uint32_t xp0 = __shfl_up(x0, 1), xp1 = __shfl_up(x1, 1);
            const uint32_t ep0 = __shfl_up(e0, 1), ep1 = __shfl_up(e1, 1);
            uint32_t h;
            if (lane <= k) {
                h = 0u | 1u << 4;  // identity (never used: lane k+1's map is constant)
            } else if (lane == k + 1) {
                const uint32_t c = match(xk);
                h = c | c << 4;
            } else {
                const uint32_t m0 = ep0 != 0xFFFFFFFFu ? match(xp0) : 2u;
                const uint32_t m1 = ep1 != 0xFFFFFFFFu ? match(xp1) : 2u;
                h = m0 | m1 << 4;
            }
#pragma unroll
            for (uint32_t d = 1; d < kWave; d <<= 1) {
                const uint32_t pv = __shfl_up(h, d);
                if (lane >= d) {  // h := h o pv
                    const uint32_t p0 = pv & 15, p1 = pv >> 4;
                    const uint32_t n0 = p0 == 2 ? 2u : p0 == 0 ? (h & 15) : (h >> 4);
                    const uint32_t n1 = p1 == 2 ? 2u : p1 == 0 ? (h & 15) : (h >> 4);
                    h = n0 | n1 << 4;
                }
            }
            const uint32_t ch = h & 15;  // lanes k+1 .. last: the chosen chain
            const bool live = lane > k && lane <= last;
            const int32_t cst = ch == 0 ? st0 : st1;
            const uint64_t errm = __ballot(live && ch < 2 && cst != LSM_OK);
            const uint32_t lim = stk != LSM_OK ? k : errm ? (uint32_t)__builtin_ctzll(errm) : last;
            const uint64_t below = lim >= kWave - 1 ? ~0ull : (2ull << lim) - 1;  // lanes <= lim
            const uint64_t missm = __ballot(live && ch == 2) & below;
            if (!missm) {
                fast = true;
                if (lane == k) {
                    acc_entry = gp;
                    acc_cnt = ck;
                } else if (live && lane <= lim) {
                    acc_entry = ch == 0 ? e0 : e1;
                    acc_cnt = ch == 0 ? c0 : c1;
                }
                const uint32_t xe = ch == 0 ? x0 : x1;
                if (lim == k) {
                    e = xk;
                    status = stk;
                } else {
                    e = uni(__builtin_amdgcn_readlane(xe, lim));
                    status = errm ? (int32_t)uni(__builtin_amdgcn_readlane((uint32_t)cst, lim)) : LSM_OK;
                }
                uint32_t t;
                wave_excl_scan(acc_cnt, &t);
                total = t;
            }
        }
        for (uint32_t l = 0; !fast && l < kWave; l++) {
            const uint32_t sl = uni(__builtin_amdgcn_readlane(ss, l));
            const uint32_t el = uni(__builtin_amdgcn_readlane(se, l));
            if (dead || sl >= el || e >= el) continue;
            uint32_t cnt, ex;
            int32_t st;
            if (l > 0 && uni(__builtin_amdgcn_readlane(e0, l)) == e) {
                cnt = uni(__builtin_amdgcn_readlane(c0, l));
                ex = uni(__builtin_amdgcn_readlane(x0, l));
                st = (int32_t)uni(__builtin_amdgcn_readlane((uint32_t)st0, l));
            } else if (l > 0 && uni(__builtin_amdgcn_readlane(e1, l)) == e) {
                cnt = uni(__builtin_amdgcn_readlane(c1, l));
                ex = uni(__builtin_amdgcn_readlane(x1, l));
                st = (int32_t)uni(__builtin_amdgcn_readlane((uint32_t)st1, l));
            } else {  // the entry share, or neither guess on the chain: chase from e
                L.chase(e, el, cnt, ex, st);
                cnt = uni(cnt);
                ex = uni(ex);
                st = (int32_t)uni((uint32_t)st);
            }
            if (lane == l) {
                acc_entry = e;
                acc_cnt = cnt;
            }
            total += cnt;
            e = ex;
            if (st != LSM_OK) {
                status = st;
                dead = true;
            }
        }
        uint32_t tot;
        const uint32_t pre = wave_excl_scan(acc_cnt, &tot);
        if (acc_cnt && !(LSM_WAL_DBG & 1)) {
            u32x4 *dst = a.scratch + q * kWalSegSlots + pre;
            uint32_t p = acc_entry;
            for (uint32_t i = 0; i < acc_cnt; i++) {
                uint32_t kl = 0, vl = 0;
                L.record(p, kl, vl);
                const uint64_t ro = off + p;
                dst[i] = u32x4{(uint32_t)ro, (uint32_t)(ro >> 32), kl, vl};
                p += 8 + kl + vl;
            }
        }
        if (lane == 0) a.seg[q] = WalSeg{gp, e, total, status};
    }
}

__global__ __launch_bounds__(64) void wal_stitch_kernel(WalArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t ring[8 * kChunk / 4 + 4];
    const uint32_t w = blockIdx.x, lane = lane_id();
    const uint32_t len = uni(a.wal_len[w]);
    const uint64_t off = uni64(a.wal_off[w]);
    uint64_t base, cap;
    wal_slots(a, w, base, cap);
    base = uni64(base);
    const uint32_t ocap = uni(cap < 0xFFFFFFFFull ? (uint32_t)cap : 0xFFFFFFFFu);
    if (len > a.max_len) {  // outside the segment grid: one exact chase, in place
        DecodeArgs d = {};
        d.in = a.wal;
        d.desc = a.out.desc ? reinterpret_cast<u32x4 *>(a.out.desc) : nullptr;
        uint32_t nr = 0;
        int32_t st = LSM_OK;
        decode_range_any<LSM_GRAMMAR_KV, 8>(d, ring, off, len, base, ocap, nr, st);
        for (uint32_t s = lane; s < a.segs; s += kWave) {
            a.fin[2 * ((uint64_t)w * a.segs + s)] = 0;
            a.fin[2 * ((uint64_t)w * a.segs + s) + 1] = 0;
        }
        if (lane == 0) {
            a.out.nrec[w] = nr;
            a.out.status[w] = st;
        }
        return;
    }
    const uint32_t nseg = (len + kWalSeg - 1) / kWalSeg;
    uint32_t e = 0, total = 0;
    int32_t status = LSM_OK;
    bool dead = false;
    for (uint32_t s0 = 0; s0 < a.segs; s0 += kWave) {
        const uint32_t sl = s0 + lane;
        const uint64_t q0 = ((uint64_t)w * a.segs + sl) * 2;
        const WalSeg T0 = sl < nseg ? a.seg[q0] : WalSeg{0, 0, 0, 0};
        const WalSeg T1 = sl < nseg ? a.seg[q0 + 1] : WalSeg{0, 0, 0, 0};
        uint32_t f_pre = 0, f_cnt = 0;
        // fast form: segment j's choice of chain (0, 1; 2 = neither, or the
        // previous chain runs past segment j's end) is a function of segment
        // j-1's choice; a 6-step scan composes these maps across the 64
        // segments of the group, as wal_seg_lanes_kernel does across shares.
        // Any miss before the first error falls back to the serial walk.
        bool fast = false;
        if (!dead && s0 < nseg) {
            const uint32_t gl = nseg - s0 < kWave ? nseg - s0 : kWave;  // live segments
            const bool live = lane < gl;
            const uint32_t send = (sl + 1) * kWalSeg;
            auto match = [&](uint32_t x) -> uint32_t {
                return x >= send ? 2u : x == T0.entry ? 0u : x == T1.entry ? 1u : 2u;
            };
            const uint32_t xp0 = __shfl_up(T0.exit, 1), xp1 = __shfl_up(T1.exit, 1);
            uint32_t h;
            if (lane == 0) {
                const uint32_t c = match(e);
                h = c | c << 4;
            } else {
                h = match(xp0) | match(xp1) << 4;
            }
#pragma unroll
            for (uint32_t d = 1; d < kWave; d <<= 1) {
                const uint32_t pv = __shfl_up(h, d);
                if (lane >= d) {  // h := h o pv
                    const uint32_t p0 = pv & 15, p1 = pv >> 4;
                    const uint32_t n0 = p0 == 2 ? 2u : p0 == 0 ? (h & 15) : (h >> 4);
                    const uint32_t n1 = p1 == 2 ? 2u : p1 == 0 ? (h & 15) : (h >> 4);
                    h = n0 | n1 << 4;
                }
            }
            const uint32_t ch = h & 15;
            const int32_t cst = ch == 0 ? T0.status : T1.status;
            const uint64_t errm = __ballot(live && ch < 2 && cst != LSM_OK);
            const uint32_t lim = errm ? (uint32_t)__builtin_ctzll(errm) : gl - 1;
            const uint64_t below = lim >= kWave - 1 ? ~0ull : (2ull << lim) - 1;  // lanes <= lim
            if (!(__ballot(live && ch == 2) & below)) {
                fast = true;
                const bool take = live && lane <= lim;
                const uint32_t nr = take ? (ch == 0 ? T0.nrec : T1.nrec) : 0u;
                const uint32_t xe = ch == 0 ? T0.exit : T1.exit;
                uint32_t sum;
                f_pre = total + wave_excl_scan(nr, &sum);
                f_cnt = nr | (take && ch == 1 ? 0x80000000u : 0u);
                total += uni(sum);
                e = uni(__builtin_amdgcn_readlane(xe, lim));
                if (errm) {
                    status = (int32_t)uni(__builtin_amdgcn_readlane((uint32_t)cst, lim));
                    dead = true;
                }
            }
        }
        for (uint32_t j = 0; !fast && j < kWave && s0 + j < nseg; j++) {
            const uint32_t s = s0 + j;
            uint32_t pre = total, cnt = 0;
            if (!dead && e < len && e < (s + 1) * kWalSeg) {
                const uint32_t e0 = uni(__builtin_amdgcn_readlane(T0.entry, j));
                const uint32_t e1 = uni(__builtin_amdgcn_readlane(T1.entry, j));
                const uint32_t ph = e0 == e ? 0u : e1 == e ? 1u : 2u;
                uint32_t ex, nr;
                int32_t st;
                if (ph == 0) {
                    ex = uni(__builtin_amdgcn_readlane(T0.exit, j));
                    nr = uni(__builtin_amdgcn_readlane(T0.nrec, j));
                    st = (int32_t)uni(__builtin_amdgcn_readlane((uint32_t)T0.status, j));
                } else if (ph == 1) {
                    ex = uni(__builtin_amdgcn_readlane(T1.exit, j));
                    nr = uni(__builtin_amdgcn_readlane(T1.nrec, j));
                    st = (int32_t)uni(__builtin_amdgcn_readlane((uint32_t)T1.status, j));
                } else {  // both guesses missed: chase from the true position
                    DecodeArgs d = {};
                    d.in = a.wal;
                    d.desc = a.scratch;
                    const uint32_t stop = ((s + 1) * kWalSeg < len ? (s + 1) * kWalSeg : len) - e;
                    uint32_t endp = 0;
                    nr = 0;
                    st = LSM_OK;
                    decode_range_any<LSM_GRAMMAR_KV, 8>(
                        d, ring, off + e, len - e, ((uint64_t)w * a.segs + s) * 2 * kWalSegSlots,
                        kWalSegSlots, nr, st, stop, &endp);
                    ex = e + endp;
                }
                cnt = nr | (ph == 1 ? 0x80000000u : 0u);
                total += nr;
                e = ex;
                if (st != LSM_OK) {
                    status = st;
                    dead = true;
                }
            } else if (e >= len) {
                dead = true;
            }
            if (lane == j) {
                f_pre = pre;
                f_cnt = cnt;
            }
        }
        if (sl < a.segs) {
            a.fin[2 * ((uint64_t)w * a.segs + sl)] = f_pre;
            a.fin[2 * ((uint64_t)w * a.segs + sl) + 1] = f_cnt;
        }
    }
    if (lane == 0) {
        if (total > ocap) {  // caller's record capacity (not a reference error)
            total = ocap;
            status = LSM_ST_CAPACITY;
        }
        a.out.nrec[w] = total;
        a.out.status[w] = status;
    }
}

__global__ __launch_bounds__(256) void wal_compact_kernel(WalArgs a) {
    const uint32_t s = blockIdx.x, w = blockIdx.y;
    const uint64_t q = (uint64_t)w * a.segs + s;
    const uint32_t pre = a.fin[2 * q], cf = a.fin[2 * q + 1];
    const uint32_t cnt = cf & 0x7FFFFFFFu;
    if (cnt == 0) return;
    uint64_t base, cap;
    wal_slots(a, w, base, cap);
    u32x4 *dst = reinterpret_cast<u32x4 *>(a.out.desc);
    const u32x4 *src = a.scratch + (q * 2 + (cf >> 31)) * kWalSegSlots;
    for (uint32_t j = threadIdx.x; j < cnt; j += blockDim.x)
        if ((uint64_t)pre + j < cap) dst[base + pre + j] = src[j];
}

}  // namespace
}  // namespace lsm

using namespace lsm;

namespace lsm {
// exclusive scan of u32 values into n + 1 u64 sums (for merge.hip)
int scan_u32_to_u64(const uint32_t *d_len, uint32_t n, uint64_t *d_out, void *ws, size_t ws_bytes,
                    hipStream_t s) {
    return plan_scan(3, d_len, n, d_out, ws, ws_bytes, s);
}
size_t scan_workspace_bytes(uint32_t n) {
    const size_t ntiles = (n + kScanTile - 1) / kScanTile;
    return (ntiles ? ntiles : 1) * 8;
}
}  // namespace lsm

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
    a.split = 0;
    static const uint32_t dbg = [] {
        const char *e = getenv("LSM_DECODE_DBG");
        return e ? (uint32_t)atoi(e) : 0u;
    }();
    a.dbg = dbg;
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


extern "C" size_t lsm_wal_replay_workspace_bytes(uint32_t nwal, uint32_t max_wal_len) {
    const uint64_t segs = max_wal_len ? ((uint64_t)max_wal_len + kWalSeg - 1) / kWalSeg : 1;
    const uint64_t n = (uint64_t)nwal * segs;
    return (size_t)(n * (2 * sizeof(WalSeg) + 8 + 2ull * kWalSegSlots * 16) + 64);
}

extern "C" int lsm_wal_replay(lsm_ctx *ctx, const uint8_t *d_wal, const uint64_t *d_wal_off,
                              const uint32_t *d_wal_len, uint32_t nwal, uint32_t max_wal_len,
                              const lsm_decode_out *out, void *d_workspace, size_t ws_bytes,
                              void *stream) {
    if (!ctx || !out) return LSM_EINVAL;
    if (nwal == 0) return 0;
    if (!d_wal || !d_wal_off || !d_wal_len || !out->desc || !out->nrec || !out->status ||
        !d_workspace || out->key_arena || out->val_arena || nwal > 65535)
        return LSM_EINVAL;
    if (ws_bytes < lsm_wal_replay_workspace_bytes(nwal, max_wal_len)) return LSM_ESPACE;
    WalArgs a;
    a.wal = d_wal;
    a.wal_off = d_wal_off;
    a.wal_len = d_wal_len;
    a.nwal = nwal;
    a.max_len = max_wal_len;
    a.segs = max_wal_len ? (max_wal_len + kWalSeg - 1) / kWalSeg : 1;
    a.out = *out;
    const uint64_t n = (uint64_t)nwal * a.segs;
    uint8_t *ws = static_cast<uint8_t *>(d_workspace);
    a.scratch = reinterpret_cast<u32x4 *>(ws);  // 16-byte aligned first
    a.seg = reinterpret_cast<WalSeg *>(ws + n * 2 * kWalSegSlots * 16);
    a.fin = reinterpret_cast<uint32_t *>(ws + n * 2 * (kWalSegSlots * 16 + sizeof(WalSeg)));
    hipStream_t s = static_cast<hipStream_t>(stream);
    static const char *wk = getenv("LSM_WAL_KERNEL");
    if (wk && !strcmp(wk, "serial"))
        hipLaunchKernelGGL(wal_seg_kernel, dim3(2 * a.segs, nwal), dim3(kWave), 0, s, a);
    else if (wk && !strcmp(wk, "lanes"))  // shares read through the caches, no LDS copy
        hipLaunchKernelGGL(wal_seg_lanes_kernel<0>, dim3(a.segs, nwal), dim3(kWave), 0, s, a);
    else if (wk && !strcmp(wk, "stage4k"))
        hipLaunchKernelGGL(wal_seg_lanes_kernel<kWalStage4k>, dim3(a.segs, nwal), dim3(kWave), 0, s, a);
    else
        hipLaunchKernelGGL(wal_seg_lanes_kernel<kWalStage>, dim3(a.segs, nwal), dim3(kWave), 0, s, a);
    hipLaunchKernelGGL(wal_stitch_kernel, dim3(nwal), dim3(kWave), 0, s, a);
    hipLaunchKernelGGL(wal_compact_kernel, dim3(a.segs, nwal), dim3(256), 0, s, a);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}

extern "C" size_t lsm_decode_sst_workspace_bytes(uint32_t nfile) {
    return (size_t)nfile * (sizeof(SstWork) + 8) + 16;
}

extern "C" int lsm_decode_sst(lsm_ctx *ctx, const uint8_t *d_img, const uint64_t *d_file_off,
                              const uint64_t *d_file_len, uint32_t nfile,
                              const uint64_t *d_rec_base, lsm_sst_meta *d_meta,
                              lsm_rec_desc *d_idx_desc, int64_t *d_idx_value,
                              lsm_rec_desc *d_data_desc, void *d_workspace, size_t ws_bytes,
                              void *stream) {
    if (!ctx) return LSM_EINVAL;
    if (nfile == 0) return 0;
    if (nfile > 65535 || !d_img || !d_file_off || !d_file_len || !d_meta || !d_idx_desc ||
        !d_idx_value || !d_data_desc || !d_workspace)
        return LSM_EINVAL;
    if (ws_bytes < lsm_decode_sst_workspace_bytes(nfile)) return LSM_ESPACE;
    hipStream_t s = static_cast<hipStream_t>(stream);
    SstArgs a;
    a.img = d_img;
    a.file_off = d_file_off;
    a.file_len = d_file_len;
    a.nfile = nfile;
    a.rec_base = d_rec_base;
    a.meta = d_meta;
    a.idx_desc = reinterpret_cast<u32x4 *>(d_idx_desc);
    a.idx_value = d_idx_value;
    a.data_desc = reinterpret_cast<u32x4 *>(d_data_desc);
    a.work = static_cast<SstWork *>(d_workspace);
    a.fail = reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(d_workspace) +
                                          (size_t)nfile * sizeof(SstWork));
    LSM_HIP_CHECK(hipMemsetAsync(a.fail, 0xFF, (size_t)nfile * 8, s));
    // parallel passes: ~kSstWgs workgroups over the batch, at most 64 per file
    static const uint32_t kSstWgs = getenv("LSM_SST_WGS") ? (uint32_t)atoi(getenv("LSM_SST_WGS")) : 2048;
    uint32_t g = (kSstWgs + nfile - 1) / nfile;
    if (g > 64) g = 64;
    if (g == 0) g = 1;
    hipLaunchKernelGGL(sst_index_kernel, dim3(g, nfile), dim3(256), 0, s, a);
    hipLaunchKernelGGL(sst_index_fixup_kernel, dim3(nfile), dim3(kWave), 0, s, a);
    hipLaunchKernelGGL(sst_data_verify_kernel, dim3(g, nfile), dim3(256), 0, s, a);
    hipLaunchKernelGGL(sst_data_fixup_kernel, dim3(nfile), dim3(kWave), 0, s, a);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}

#ifdef LSM_STAMPS
extern "C" int lsm_debug_set_stamps(void *d_buf) {
    LSM_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(lsm::g_stamps), &d_buf, sizeof(void *)));
    return 0;
}
#endif
