// decode.hip — batched record decode of length-prefixed blocks on gfx950.
//
// One wavefront (and one workgroup) owns one block: go-lsm's blocks are
// independent units, so the parallelism is across blocks.  The
// block streams through an 8 KiB per-wave LDS ring of 1 KiB chunks, loaded by
// LDS-DMA (buffer_load_dwordx4 ... lds, range-checked so a block never reads
// past its padded end).  Record boundaries are a dependent chain (each
// position depends on every earlier length, data.go:58-76): the wave verifies
// 64 records at a time by speculative runs and chases the rest exactly on
// the VALU (decode_range_v2).  Descriptors leave as coalesced 16-byte stores;
// in ARENA mode the key and value bytes are gathered from the LDS ring into
// packed arenas with 16-byte stores (the bytes Go's make()+ReadFull produce).
// Also here: the whole-.sst decode (f1), WAL replay (f4) and the dense
// compaction of decoded records.
#include <stdlib.h>
#include <string.h>

#include "common.h"

namespace lsm {
namespace {

constexpr uint32_t kChunk = 1024;  // one b128 wave-load
constexpr uint32_t kRingChunks = 8;  // 8 KiB ring: 4 KiB blocks fit whole, 64 KiB stream
// Cache policy of the block loads: nt (streaming).  Each block byte is read
// once; keeping the stream out of the L2/MALL's normal replacement measured
// 80.5 -> 71.7 us for decode4k's memory pattern (tools/block_probe.py).
constexpr int kBlockLoadAux = 2;
// Per ring size (A/B on one box, wall GiB/s: resident / rotated copies / one
// 1M-block launch): the 8 KiB ring (4 KiB blocks) stores its descriptors nt
// too: 4,800 / 4,045 / 4,100 with plain stores, 4,836 / 4,800 / 4,650 with nt
// stores.  ARENA on the 8 KiB ring also loads the blocks with the default
// policy (2,150 -> 2,290 GiB/s).  The 16 KiB ring (64 KiB blocks) and the
// 2 KiB ring (mixed, scheduled) keep plain stores: nt stores measured 4,530
// -> 4,140 and 5,030 -> 4,850 GiB/s there.
// A launch of more than kBigLaunch blocks on the 8 KiB ring (gigabytes of
// input, far past the 256 MB MALL) loads its blocks with the default policy:
// 1M blocks 4,610 -> 5,030 GiB/s, 500k 4,835 -> 4,945; at 250k and below nt
// loads stay ahead (250k: 4,880 against 4,776; 100k, resident: 4,850 against
// 4,600).
constexpr uint32_t kBigLaunch = 400000;
template <uint32_t NCH, bool ARENA, bool BIG = false>
struct RingPolicy {
    static constexpr int load_aux = ((ARENA || BIG) && NCH == 8) ? 0 : kBlockLoadAux;
    static constexpr bool nt_desc = NCH == 8;
};
template <uint32_t NCH, bool ARENA>
__device__ __forceinline__ void store_desc(u32x4 *p, const u32x4 &d) {
    if (RingPolicy<NCH, ARENA>::nt_desc)
        __builtin_nontemporal_store(d, p);
    else
        *p = d;
}


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
    const uint32_t *order;  // launch order of the blocks (null: 0, 1, ..)
};

// Streams one block through this wave's LDS ring and serves u32 length
// fields at wave-uniform block positions.
//
// Ring: NCH x 1 KiB chunks, filled by LDS-DMA (buffer_load_dwordx4 ... lds:
// no VGPR staging), read by the chase with ds_read at block positions.
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

template <uint32_t NCH, int AUX = kBlockLoadAux>
struct BlockReaderT {
    uint32_t *ring;
    rsrc_t rsrc;
    uint32_t h;        // block start inside its first 16-byte line
    uint32_t total;    // loadable stream bytes: round_up16(h + n)
    uint32_t nchunks;  // chunks covering [0, total)
    uint32_t hi_c;     // chunks [.., hi_c) have been issued into the ring
    uint32_t landed;   // chunks [.., landed) are known to be in LDS

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
                    16, voff + c * kChunk, 0, 0, AUX);
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

};
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

// ---- v2: the chase with the fewest scalar instructions -------------------
//
// The exact step is a serial chain, and a wave-uniform chain runs on the CU's
// one scalar unit, shared by all resident waves: PMC on config 5 (record
// shapes vary, so speculative runs rarely verify) counted 107 SALU
// instructions per record for the round-0 wave-uniform step, 74% of the
// kernel time at one SALU issue per cycle.  v2 keeps the same semantics with
// a leaner step:
//  * one compare decides whether the bytes are landed (`lim`), the ring
//    bookkeeping only runs when a step crosses it;
//  * blocks that fit the ring are read without modulo arithmetic (LIN);
//  * the value length is read at the previous key length in the same LDS
//    round trip as the key length;
//  * descriptors are staged branch-free (v_cndmask) and stored 64 at a time;
//  * error statuses are only computed on the (one) failing record.
// Speculative runs: after an exact step of size S (key length K, value
// length V) all 64 lanes test "the next 64 records have the same K and V"
// straight from LDS; the ballot's count of leading successes is the verified
// run (each check reads the record's own fields, so the verified records are
// exactly the chase's), stored coalesced.
// A wave-uniform value moved into a VGPR, so the arithmetic that depends on
// it stays on the vector ALU (the compiler would otherwise keep a uniform
// chain on the CU's single scalar unit).
__device__ __forceinline__ uint32_t to_vgpr(uint32_t s) {
    uint32_t v;
    __asm__ __volatile__("v_mov_b32 %0, %1" : "=v"(v) : "s"(s));
    return v;
}

// ---- ARENA: key and value bytes gathered from the LDS ring -----------------
//
// kv.go:88-111 / data.go:68-75 hand back freshly allocated key and value
// slices; ARENA mode packs them per block, in record order, into a key arena
// and a value arena.  A batch of records (a verified run, or the <= 64 staged
// records of exact steps) occupies one contiguous range of each arena, so the
// copy is output-driven: each lane assembles one 16-byte output chunk from
// the record fields it covers (four funnel-shifted dwords, bytewise only
// where a record boundary falls inside a dword) and stores it whole.  Only a
// batch's first and last chunks, shared with the neighbouring batch or
// block, are written byte by byte.
template <uint32_t NCH, bool LIN>
struct RingBytes {
    const uint32_t *ring;
    rsrc_t rs;          // the block in global memory (stream byte = rsrc offset)
    uint32_t res_lo;    // stream bytes [res_lo, res_hi) are landed in the ring
    uint32_t res_hi;
    __device__ __forceinline__ uint32_t word(uint32_t w) const {
        return LIN ? ring[w] : ring[w % (NCH * kChunk / 4)];
    }
    // the ring dword at dword-aligned stream byte sb
    __device__ __forceinline__ uint32_t word_at(uint32_t sb) const {
        constexpr uint32_t kB = NCH * kChunk;
        return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(ring) +
                                                   (LIN ? sb : sb & (kB - 1)));
    }
    __device__ __forceinline__ uint32_t u32(uint32_t sb) const {
        return funnel(word(sb >> 2), word((sb >> 2) + 1), sb);
    }
    __device__ __forceinline__ uint32_t u8(uint32_t sb) const {
        return (word(sb >> 2) >> (8 * (sb & 3))) & 0xFFu;
    }
    // stream bytes [sb, sb + 16) from two aligned 16-byte LDS lines: two
    // ds_read_b128 (conflict-free when lanes take consecutive chunks; five
    // ds_read_b32 at a 16-byte lane stride are 4-way bank conflicts)
    __device__ __forceinline__ u32x4 u128(uint32_t sb) const {
        constexpr uint32_t kB = NCH * kChunk;
        const uint32_t a = sb & ~15u;
        const uint32_t i0 = (LIN ? a : a % kB) >> 2, i1 = (LIN ? a + 16 : (a + 16) % kB) >> 2;
        const u32x4 x = *reinterpret_cast<const u32x4 *>(&ring[i0]);
        const u32x4 y = *reinterpret_cast<const u32x4 *>(&ring[i1]);
        const uint32_t d = (sb >> 2) & 3;
        const uint32_t d0 = d == 0 ? x.x : d == 1 ? x.y : d == 2 ? x.z : x.w;
        const uint32_t d1 = d == 0 ? x.y : d == 1 ? x.z : d == 2 ? x.w : y.x;
        const uint32_t d2 = d == 0 ? x.z : d == 1 ? x.w : d == 2 ? y.x : y.y;
        const uint32_t d3 = d == 0 ? x.w : d == 1 ? y.x : d == 2 ? y.y : y.z;
        const uint32_t d4 = d == 0 ? y.x : d == 1 ? y.y : d == 2 ? y.z : y.w;
        return u32x4{funnel(d0, d1, sb), funnel(d1, d2, sb), funnel(d2, d3, sb),
                     funnel(d3, d4, sb)};
    }
    // a field not (wholly) in the ring: read through the caches
    __device__ __forceinline__ uint32_t g32(uint32_t sb) const {
        const uint32_t a = sb & ~3u;
        return funnel(ld_b32(rs, a), ld_b32(rs, a + 4), sb);
    }
    __device__ __forceinline__ uint32_t g8(uint32_t sb) const {
        return (ld_b32(rs, sb & ~3u) >> (8 * (sb & 3))) & 0xFFu;
    }
};

// Store 16 bytes at the 16-aligned dst; only bytes [lo, hi) are this batch's
// (a batch's first and last chunk share 16 bytes with its neighbours).  The
// arena streams are written once: every arena store is nt (A/B, config 2
// ARENA: 160-168 -> 145-146 us per launch).
__device__ __forceinline__ void store_chunk(uint8_t *dst, u32x4 v, int lo, int hi) {
    if (lo <= 0 && hi >= 16) {
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(dst));
        return;
    }
#pragma unroll 1
    for (int t = lo < 0 ? 0 : lo; t < (hi < 16 ? hi : 16); t++) {
        const uint32_t d = t < 4 ? v.x : t < 8 ? v.y : t < 12 ? v.z : v.w;
        dst[t] = (uint8_t)(d >> (8 * (t & 3)));
    }
}

__device__ __forceinline__ void set_dword(u32x4 &v, uint32_t j, uint32_t w) {
    v.x = j == 0 ? w : v.x;
    v.y = j == 1 ? w : v.y;
    v.z = j == 2 ? w : v.z;
    v.w = j == 3 ? w : v.w;
}

// A verified run: cnt records of stride S whose field of L bytes starts at
// ring stream byte src0 + i*S (all landed), packed to out[0, cnt*L).  One
// output dword per lane per step (consecutive lanes read consecutive ring
// dwords: no bank conflicts; 256-byte coalesced stores), with as few VALU
// operations per dword
// as the shape allows: the field index by one FMA (q / L rounded from
// q + 1/2, exact for q < 2^16), the second ring dword only where some lane's
// source is unaligned, the next field's bytes only where a field boundary
// falls inside some lane's dword (k < 4), bytes singly only in the run's
// first and last dword.  Ring reads are indexed modulo the ring, so lanes
// past the end read harmless bytes.
// a*b + c for a, b < 2^24 (full-rate v_mad_u32_u24; b wave-uniform)
__device__ __forceinline__ uint32_t mad_u24(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    __asm__("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(d) : "v"(a), "s"(b), "v"(c));
    return d;
}

template <uint32_t NCH, bool LIN>
__device__ __forceinline__ void arena_emit_run(const RingBytes<NCH, LIN> &rb, uint8_t *out,
                                               uint32_t src0, uint32_t S, uint32_t L,
                                               uint32_t cnt) {
    const uint32_t T = cnt * L;  // <= the ring: a run lies inside the landed bytes
    if (T == 0) return;
    const uint32_t lane = lane_id();
    // full-rate 24-bit products (v_mul_u32_u24): every operand here is < 2^24
    auto mul24 = [](uint32_t x, uint32_t y) { return (x & 0xFFFFFFu) * (y & 0xFFFFFFu); };
    if (((src0 | S | L | (uint32_t)(uintptr_t)out) & 3) == 0) {
        // dword-aligned run: output dword j is ring byte src0 + 4j + r*(S-L)
        // with r = floor(j / (L/4)) -- one ring read and one store per dword.
        // The stores go through a buffer resource spanning exactly the run:
        // lanes past its end are dropped by the range check (no exec masks,
        // no 64-bit address arithmetic; the whole offset is in the VGPR).
        const uint32_t L4 = L >> 2, GB = S - L;
        // floor((j + 1/2) * rcp(L4)) is exact for j < 2^16: the quotient is at
        // least 1/(2 L4) from an integer, the error below 2^-6 / L4
        const float inv4 = __builtin_amdgcn_rcpf((float)L4), hinv4 = 0.5f * inv4;
        const rsrc_t os = make_rsrc(out, T);
        constexpr uint32_t V = 4;  // ring reads in flight per lane
#pragma unroll 1
        for (uint32_t b = 0; b < T; b += 4 * V * kWave) {  // wave-uniform output byte
            uint32_t v[V], o[V];
#pragma unroll
            for (uint32_t t = 0; t < V; t++) {  // past the run: harmless ring bytes
                const uint32_t j = (b >> 2) + t * kWave + lane;
                const uint32_t r = (uint32_t)__builtin_fmaf((float)j, inv4, hinv4);
                o[t] = 4 * j;
                v[t] = rb.word_at(mad_u24(r, GB, src0 + o[t]));
            }
#pragma unroll
            for (uint32_t t = 0; t < V; t++) __builtin_amdgcn_raw_buffer_store_b32(v[t], os, o[t], 0, 2);
        }
        return;
    }
    const uint32_t lead = (uint32_t)((uintptr_t)out & 3);
    uint32_t *a0 = reinterpret_cast<uint32_t *>(out - lead);
    const uint32_t nd = (lead + T + 3) >> 2;
    const float inv = 1.0f / (float)L, hinv = 0.5f * inv;  // once per run
    auto rec = [&](uint32_t q) -> uint32_t {  // floor(q / L), q < 2^16
        return (uint32_t)__builtin_fmaf((float)q, inv, hinv);
    };
    constexpr uint32_t U = 1;  // dwords per lane per step (2 and 4 measured no faster)
#pragma unroll 1
    for (uint32_t w0 = 0; w0 < nd; w0 += U * kWave) {
        uint32_t W[U], sb[U], kk[U], rr[U];
        int qv[U];
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const int q = (int)(4 * (w0 + u * kWave + lane)) - (int)lead;
            const uint32_t qc = q < 0 ? 0u : (uint32_t)q;
            const uint32_t r = rec(qc), o = qc - mul24(r, L);
            qv[u] = q;
            rr[u] = r;
            kk[u] = L - o;
            sb[u] = src0 + mul24(r, S) + o;
            W[u] = rb.word(sb[u] >> 2);
        }
        bool unal = false, cross = false;
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            unal |= (sb[u] & 3) != 0;
            cross |= kk[u] < 4;
        }
        if (__ballot(unal)) {
#pragma unroll
            for (uint32_t u = 0; u < U; u++) W[u] = funnel(W[u], rb.word((sb[u] >> 2) + 1), sb[u]);
        }
        if (L < 4) {  // fields of 0-3 bytes: byte by byte
#pragma unroll
            for (uint32_t u = 0; u < U; u++) {
                const uint32_t qc = qv[u] < 0 ? 0u : (uint32_t)qv[u];
                uint32_t x = 0;
                for (uint32_t t = 0; t < 4; t++) {
                    const uint32_t qq = qc + t;
                    if (qq < T) {
                        const uint32_t r = rec(qq);
                        x |= rb.u8(src0 + mul24(r, S) + (qq - mul24(r, L))) << (8 * t);
                    }
                }
                W[u] = x;
            }
        } else if (__ballot(cross)) {  // a field boundary inside some lane's dword
#pragma unroll
            for (uint32_t u = 0; u < U; u++) {
                const uint32_t B = rb.u32(src0 + mul24(rr[u] + 1, S)), k = kk[u];
                W[u] = k < 4 ? (W[u] & ((1u << (8 * k)) - 1)) | (B << (8 * k)) : W[u];
            }
        }
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint32_t w = w0 + u * kWave + lane;
            const int q = qv[u];
            if (q >= 0 && (uint32_t)q + 4 <= T) {
                __builtin_nontemporal_store(W[u], &a0[w]);
            } else if (w < nd) {  // the run's first or last dword, shared with its neighbours
                const uint32_t sh = q < 0 ? (uint32_t)(-q) : 0u;  // bytes before the run
                uint8_t *b = reinterpret_cast<uint8_t *>(a0 + w);
                for (uint32_t t = sh; t < 4 && (uint32_t)(q + (int)t) < T; t++)
                    b[t] = (uint8_t)(W[u] >> (8 * (t - sh)));
            }
        }
    }
}

// A staged batch: lane l < cnt holds a record field of len bytes at ring
// stream byte src; the fields are packed in lane order to out[0, T).  A field
// wholly landed in the ring is read from LDS, any other (a value longer than
// the ring) through the caches.  tab: 129 dwords of LDS.  Returns T.
template <uint32_t NCH, bool LIN>
__device__ __forceinline__ uint32_t arena_emit_batch(const RingBytes<NCH, LIN> &rb, uint32_t *tab,
                                                     uint8_t *out, uint32_t cnt, uint32_t src,
                                                     uint32_t len, uint64_t *out_off,
                                                     uint64_t cur) {
    const uint32_t lane = lane_id();
    const uint32_t l = lane < cnt ? len : 0u;
    uint32_t T;
    const uint32_t start = wave_excl_scan(l, &T);
    if (out_off && lane < cnt) out_off[lane] = cur + start;
    if (T == 0) return 0;
    uint32_t *tstart = tab, *tsrc = tab + 65;
    if (lane < cnt) {
        tstart[lane] = start;
        tsrc[lane] = src;
    }
    if (lane == 0) tstart[cnt] = T;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t lead = (uint32_t)((uintptr_t)out & 15);
    uint8_t *a0 = out - lead;
    const uint32_t nch = (lead + T + 15) >> 4;
#pragma unroll 1
    for (uint32_t c = lane; c < nch; c += kWave) {
        const int q0 = (int)(16 * c) - (int)lead;
        const uint32_t qf = q0 < 0 ? 0u : (uint32_t)q0;
        // the last record whose packed range starts at or before qf
        uint32_t lo = 0, hi = cnt;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (tstart[mid] <= qf) lo = mid;
            else hi = mid;
        }
        uint32_t r = lo, rs0 = tstart[r], rs1 = tstart[r + 1], rsrc = tsrc[r];
        auto in_ring = [&]() { return rsrc >= rb.res_lo && rsrc + (rs1 - rs0) <= rb.res_hi; };
        auto seek = [&](uint32_t q) {  // advance r to the record holding byte q
            while (rs1 <= q) {
                r++;
                rs0 = rs1;
                rs1 = tstart[r + 1];
                rsrc = tsrc[r];
            }
        };
        auto byte_at = [&](uint32_t q) -> uint32_t {
            seek(q);
            const uint32_t sb = rsrc + (q - rs0);
            return in_ring() ? rb.u8(sb) : rb.g8(sb);
        };
        u32x4 v{0, 0, 0, 0};
        if (q0 >= 0 && q0 + 16 <= (int)T && (uint32_t)q0 + 16 <= rs1) {
            // the chunk lies in one field
            const uint32_t sb = rsrc + ((uint32_t)q0 - rs0);
            if (in_ring())
                v = rb.u128(sb);
            else
                v = u32x4{rb.g32(sb), rb.g32(sb + 4), rb.g32(sb + 8), rb.g32(sb + 12)};
        } else {
#pragma unroll 1
            for (int t = 0; t < 16; t++) {
                const int q = q0 + t;
                if (q >= 0 && q < (int)T) {
                    const uint32_t b = byte_at((uint32_t)q) << (8 * (t & 3));
                    set_dword(v, (uint32_t)t >> 2, (t < 4 ? v.x : t < 8 ? v.y : t < 12 ? v.z : v.w) | b);
                }
            }
        }
        store_chunk(a0 + 16 * c, v, -q0, (int)T - q0);
    }
    // the table is rewritten by the next batch: all reads done first
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return T;
}

typedef __attribute__((address_space(3))) uint32_t lds_u32_t;

// arena_emit_batch as one out-of-line call per batch: a staged flush has
// several call sites in the chase, and inlining each multiplies the live
// registers of the whole kernel.  The LDS pointers keep their address space
// (ds_read, not flat loads).
template <uint32_t NCH, bool LIN>
__device__ __forceinline__ uint32_t arena_emit_batch_call(lds_u32_t *ring, rsrc_t rs, uint32_t res_lo,
                                                       uint32_t res_hi, lds_u32_t *tab,
                                                       uint8_t *out, uint32_t cnt, uint32_t src,
                                                       uint32_t len, uint64_t *out_off,
                                                       uint64_t cur) {
    RingBytes<NCH, LIN> rb{(const uint32_t *)ring, rs, res_lo, res_hi};
    return arena_emit_batch(rb, (uint32_t *)tab, out, cnt, src, len, out_off, cur);
}

// Arena cursors of one block (ARENA mode): the next free byte of each arena.
struct ArenaCur {
    uint64_t k, v;
};

// Decode the byte range [off, off + n) of a.in as one block whose records
// go to slots base.. (capacity ncap); returns the record count, the status
// and the position where the chase stopped.  Records that start at or past
// `stop` are not decoded (a clean stop; stop = n decodes the whole range).
// ARENA: keys and values are also packed into a.key_arena / a.val_arena from
// the cursors `ac` (tab: the 129-dword LDS table of arena_emit_batch).
template <int G, uint32_t NCH, bool LIN, bool ARENA = false, bool BIG = false>
__device__ void decode_range_v2(const DecodeArgs &a, uint32_t *ring, uint64_t off, uint32_t n,
                                uint64_t base, uint32_t ncap, uint32_t &nr_out, int32_t &st_out,
                                uint32_t stop, uint32_t &pos_out, ArenaCur ac = {},
                                uint32_t *tab = nullptr, bool lin_rt = LIN) {
    // the block fits the ring (read linearly, landed whole at the first
    // step): a template constant, or for ARENA a runtime flag (the ring is
    // then always indexed modulo its size, which is the same for such blocks)
    const bool lin = ARENA ? lin_rt : LIN;
    const uint32_t lane = lane_id();
    BlockReaderT<NCH, RingPolicy<NCH, ARENA, BIG>::load_aux> rd;
    rd.init(ring, a.in, off, n);
    RingBytes<NCH, LIN> rb{ring, rd.rsrc, 0, 0};

    auto word = [&](uint32_t w) -> uint32_t { return rb.word(w); };
    auto fld = [&](uint32_t p) -> uint32_t {  // wave-uniform u32 at block position p
        return uni(rb.u32(rd.h + p));
    };
    auto lds_u32 = [&](uint32_t p) -> uint32_t {  // per-lane u32 at block position p
        return rb.u32(rd.h + p);
    };

    uint32_t s_pos = 0, s_k = 0, s_v = 0, s_xlo = 0, s_xhi = 0, ns = 0, s_first = 0;
    uint32_t pos = 0, nr = 0, kprev = 0xFFFFFFFFu, miss = 0, skip = 0;
    // ARENA: the exact step's record (the last staged one) leaves its arena
    // bytes together with the run that follows it (same K, V, stride)
    uint32_t pend = 0, pend_pos = 0, pend_k = 0, pend_v = 0;
    auto emit_run_arena = [&](uint32_t p0, uint32_t K, uint32_t V, uint32_t S, uint32_t cnt,
                              uint64_t slot0) {
        // keys, then values: one emitter body serves both arenas
#pragma unroll 1
        for (uint32_t f = G == LSM_GRAMMAR_V ? 1u : 0u; f < (G == LSM_GRAMMAR_IDX ? 1u : 2u);
             f++) {
            uint8_t *ar = f ? a.val_arena : a.key_arena;
            if (!ar) continue;
            uint64_t *ao = f ? a.val_arena_off : a.key_arena_off;
            const uint64_t cur = f ? ac.v : ac.k;
            const uint32_t L = f ? V : K;
            arena_emit_run(rb, ar + cur, rd.h + p0 + (f == 0 ? 4u : G == LSM_GRAMMAR_KV ? 8 + K : 4u),
                           S, L, cnt);
            if (ao)  // cnt <= 65: the pending record + a full run
                for (uint32_t i = lane; i < cnt; i += kWave) ao[slot0 + i] = cur + (uint64_t)i * L;
            if (f) ac.v += (uint64_t)cnt * L;
            else ac.k += (uint64_t)cnt * L;
        }
    };
    auto flush = [&]() {
        if (ns) {
            if (lane < ns) {
                const uint64_t ro = off + s_pos;
                u32x4 d;
                d.x = (uint32_t)ro;
                d.y = (uint32_t)(ro >> 32);
                d.z = s_k;
                d.w = s_v;
                store_desc<NCH, ARENA>(&a.desc[base + s_first + lane], d);
                if (G == LSM_GRAMMAR_IDX && a.idx_value)
                    a.idx_value[base + s_first + lane] = (int64_t)((uint64_t)s_xhi << 32 | s_xlo);
            }
            if (ARENA && ns > pend) {  // (the pending record leaves with its run)
                lds_u32_t *lring = (lds_u32_t *)ring, *ltab = (lds_u32_t *)tab;
                // keys, then values: one emitter body serves both arenas
#pragma unroll 1
                for (uint32_t f = G == LSM_GRAMMAR_V ? 1u : 0u;
                     f < (G == LSM_GRAMMAR_IDX ? 1u : 2u); f++) {
                    uint8_t *ar = f ? a.val_arena : a.key_arena;
                    if (!ar) continue;
                    uint64_t *ao = f ? a.val_arena_off : a.key_arena_off;
                    const uint64_t cur = f ? ac.v : ac.k;
                    const uint32_t src =
                        rd.h + s_pos + (f == 0 ? 4u : G == LSM_GRAMMAR_KV ? 8 + s_k : 4u);
                    const uint32_t t = arena_emit_batch_call<NCH, LIN>(
                        lring, rb.rs, rb.res_lo, rb.res_hi, ltab, ar + cur, ns - pend, src,
                        f ? s_v : s_k, ao ? ao + base + s_first : nullptr, cur);
                    if (f) ac.v += t;
                    else ac.k += t;
                }
            }
            ns = 0;
        }
    };
    // Block bytes below `lim` (and at or above the last anchor) are landed.
    uint32_t lim = 0;
    auto need = [&](uint32_t p, uint32_t len) {
        if ((uint64_t)p + len <= lim) return;
        // a streamed block recycles ring chunks: the staged records' arena
        // bytes leave first
        if (ARENA && !lin) {
            flush();
            if (pend) {
                emit_run_arena(pend_pos, pend_k, pend_v, 0, 1, base + nr - 1);
                pend = 0;
            }
        }
        rd.ensure(rd.h + p, lin ? rd.total : len);
        lim = rd.landed >= rd.nchunks ? n : rd.landed * kChunk - rd.h;
        if (ARENA) {
            rb.res_lo = (rd.hi_c > NCH ? rd.hi_c - NCH : 0u) * kChunk;
            rb.res_hi = rd.landed * kChunk;
        }
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
        nr++;
        pos += S;

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
        // the exact record is still staged (not flushed as a 64th) and wholly
        // in the ring (landed, and its start not recycled by the value-length
        // refill of a streamed block)
        if (ARENA && ns > 0 && pos <= lim && rd.h + pos - S >= rb.res_lo) {
            pend = 1;
            pend_pos = pos - S;
            pend_k = K;
            pend_v = V;
        }
        flush();
        for (bool first = true;; first = false) {
            if (pos >= n) break;
            // wait for the span the run can verify (64 records): all of a
            // block that fits the ring, half the ring otherwise (the other
            // half stays in flight while the run is checked)
            const uint32_t span_max = (lin ? NCH : NCH / 2) * kChunk;
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
                store_desc<NCH, ARENA>(&a.desc[base + nr + lane], d);
                if (G == LSM_GRAMMAR_IDX && a.idx_value) a.idx_value[base + nr + lane] = (int64_t)xx;
            }
            if (ARENA && j + pend) {
                // the run's fields (and the pending exact record's, S bytes
                // before it) are landed: straight from the ring
                emit_run_arena(pos - pend * S, K, V, S, j + pend, base + nr - pend);
                pend = 0;
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
            // a run cut short by the landed limit goes on once more bytes
            // have landed (no exact step in between); a mismatch ends it
            if (j < 64 && !(at_lim && j > 0)) break;
        }
        if (ARENA && pend) {  // no run followed (the block ended)
            emit_run_arena(pend_pos, pend_k, pend_v, 0, 1, base + nr - 1);
            pend = 0;
        }
    }
    flush();
    nr_out = nr;
    st_out = status;
    pos_out = pos;
}

template <int G, uint32_t NCH, bool LIN, bool ARENA, bool BIG = false>
__device__ void decode_block_v2(const DecodeArgs &a, uint32_t b, uint32_t *ring, uint32_t *tab,
                                uint64_t off, uint32_t n, bool lin_rt = LIN) {
    uint64_t base, cap;
    record_slots<G>(a, b, off, n, base, cap);
    uint32_t nr, end;
    int32_t st;
    ArenaCur ac{};
    if (ARENA) {  // A(b): arena_base[b], or offset-addressed arenas
        ac.k = a.arena_base ? uni64(a.arena_base[b]) : off;
        ac.v = ac.k;
    }
    decode_range_v2<G, NCH, LIN, ARENA, BIG>(a, ring, off, n, uni64(base),
                                        uni(cap < 0xFFFFFFFFull ? (uint32_t)cap : 0xFFFFFFFFu), nr,
                                        st, n, end, ac, tab, lin_rt);
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
template <int G, uint32_t NCH, bool ARENA, bool BIG = false>
__global__ __launch_bounds__(64) void decode_v2_kernel(DecodeArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t ring[NCH * kChunk / 4 + 4];
    __shared__ uint32_t tab[ARENA ? 129 : 1];
    // a caller's launch order (largest first) is kept as given.  Large blocks
    // (the 16 KiB ring) go XCD-contiguous: 64 KiB blocks 87.9 -> 86.2 us.
    // Small blocks keep the dispatch order: XCD-contiguous 4 KiB blocks
    // measured 76.7 -> 80.0 us (eight separate address streams; the chip
    // streams one interleaved window faster).
    const uint32_t b = a.order ? uni(a.order[blockIdx.x])
                               : NCH >= 16 ? xcd_linear(blockIdx.x, a.nblk) : blockIdx.x;
    const uint64_t off = uni64(a.blk_off[b]);
    const uint32_t n = uni(a.blk_len[b]);
    const bool lin = ((off & 15) + (uint64_t)n + 15) / 16 * 16 <= NCH * kChunk;
    if (ARENA) {
        // one instantiation, the ring form a runtime flag: with both forms
        // inlined the register allocator needs 248 VGPRs (and spills) for
        // what each alone does in 96
        decode_block_v2<G, NCH, false, true>(a, b, ring, tab, off, n, lin);
    } else if (lin) {
        decode_block_v2<G, NCH, true, false, BIG>(a, b, ring, tab, off, n);
    } else {
        decode_block_v2<G, NCH, false, false, BIG>(a, b, ring, tab, off, n);
    }
}

// ---- planning: exclusive scans over per-block quantities -----------------

constexpr uint32_t kScanThreads = 256;
constexpr uint32_t kScanPer = 2;  // 16 (lanes 128 B apart) measured 1% slower on the compaction
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

// one pass over the tile sums by 1,024 threads: each a contiguous stretch of
// them (its loads in flight together), one block scan of the stretch sums (a
// loop of 256-thread block scans over 256-tile chunks took 16 us for 6,400
// tiles: a round trip per chunk)
constexpr uint32_t kPartThreads = 1024;

__global__ __launch_bounds__(kPartThreads) void plan_scan_partials(uint64_t *partial,
                                                                   uint32_t ntiles, uint64_t *out,
                                                                   uint32_t n) {
    __shared__ uint64_t wsum[kPartThreads / kWave];
    const uint32_t per = (ntiles + kPartThreads - 1) / kPartThreads, b = threadIdx.x * per;
    const uint32_t e = b + per < ntiles ? b + per : ntiles;
    uint64_t s = 0;
    for (uint32_t i0 = b; i0 < e; i0 += 8) {
        uint64_t v[8];
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) v[k] = i0 + k < e ? partial[i0 + k] : 0;
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) s += v[k];
    }
    uint64_t wt;
    const uint64_t wx = wave_excl_scan64(s, &wt);
    const uint32_t w = threadIdx.x / kWave;
    if (lane_id() == 0) wsum[w] = wt;
    __syncthreads();
    uint64_t pre = wx, tot = 0;
    for (uint32_t i = 0; i < kPartThreads / kWave; i++) {
        pre += i < w ? wsum[i] : 0;
        tot += wsum[i];
    }
    for (uint32_t i0 = b; i0 < e; i0 += 8) {
        uint64_t v[8];
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) v[k] = i0 + k < e ? partial[i0 + k] : 0;
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) {
            if (i0 + k < e) partial[i0 + k] = pre;
            pre += v[k];
        }
    }
    if (threadIdx.x == 0) out[n] = tot;
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
    hipLaunchKernelGGL(plan_scan_partials, dim3(1), dim3(kPartThreads), 0, s, partial, ntiles,
                       d_out, n);
    hipLaunchKernelGGL(plan_tile_apply, dim3(ntiles), dim3(kScanThreads), 0, s, mode, d_len, n,
                       partial, d_out);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}

template <int G, bool ARENA, uint32_t NCH = kRingChunks>
int launch_decode(const DecodeArgs &a, hipStream_t s) {
    static_assert(NCH >= 2, "a record header may straddle two ring chunks");
    if (!ARENA && NCH == kRingChunks && a.nblk > kBigLaunch && !a.order)
        hipLaunchKernelGGL((decode_v2_kernel<G, NCH, false, true>), dim3(a.nblk), dim3(kWave), 0, s, a);
    else
        hipLaunchKernelGGL((decode_v2_kernel<G, NCH, ARENA>), dim3(a.nblk), dim3(kWave), 0, s, a);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}

// ---- largest-first block schedule --------------------------------------------
//
// One wave decodes one block, and a block's chase cannot be split, so a
// batch of mixed sizes ends with a tail of the large blocks dispatched last
// streaming alone at a single wave's rate (config 5: 246 us as generated,
// 175 us with the blocks sorted largest first).  lsm_decode_blocks_scheduled
// orders the launch by size class, largest first -- quarter-octave classes
// (the leading bit and the two below it), so the order is close to sorted --
// with two small kernels and no atomics outside LDS: per tile of blocks a
// class histogram, then per tile the scatter of its block ids behind the
// larger classes and behind the earlier tiles' blocks of the same class.
// Every output is addressed by block id, so the results do not depend on
// the order.
constexpr uint32_t kSchedSub = 2;  // bits below the leading one that split an octave
constexpr uint32_t kSchedClasses = (33 - kSchedSub) << kSchedSub;
constexpr uint32_t kSchedThreads = 1024;
constexpr uint32_t kSchedPer = 16;  // blocks per thread
constexpr uint32_t kSchedTile = kSchedThreads * kSchedPer;
static_assert(kSchedClasses <= kSchedThreads, "one thread per class");

__device__ __forceinline__ uint32_t size_class(uint32_t n) {
    if (n < (1u << kSchedSub)) return n;
    const uint32_t l = 31 - __clz(n);  // kSchedSub..31
    return ((l - kSchedSub + 1) << kSchedSub) | ((n >> (l - kSchedSub)) & ((1u << kSchedSub) - 1));
}

// Class counters are kept per lane (h2[c][lane]): the lanes of one LDS
// atomic never share an address (a batch has few classes, and 64 lanes on one
// counter serialize: 7.6 us for the histogram of config 5's 37k blocks).
constexpr uint32_t kSchedLaneWords = kSchedClasses * kWave;

__device__ __forceinline__ void sched_count(const uint32_t *len, uint32_t nblk, uint32_t t0,
                                            uint32_t (*h2)[kWave], uint32_t n[kSchedPer]) {
    for (uint32_t i = threadIdx.x; i < kSchedLaneWords; i += kSchedThreads) (&h2[0][0])[i] = 0;
#pragma unroll
    for (uint32_t u = 0; u < kSchedPer; u++) {
        const uint32_t i = t0 + u * kSchedThreads;
        n[u] = i < nblk ? len[i] : 0;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t u = 0; u < kSchedPer; u++)
        if (t0 + u * kSchedThreads < nblk) atomicAdd(&h2[size_class(n[u])][lane_id()], 1u);
    __syncthreads();
}

__global__ __launch_bounds__(kSchedThreads) void sched_hist_kernel(const uint32_t *len, uint32_t nblk,
                                                                  uint32_t *hist) {
    __shared__ uint32_t h2[kSchedClasses][kWave];
    const uint32_t t0 = blockIdx.x * kSchedTile + threadIdx.x;
    uint32_t n[kSchedPer];
    sched_count(len, nblk, t0, h2, n);
    // a wave per class: the 64 lane counters summed
    for (uint32_t c = threadIdx.x / kWave; c < kSchedClasses; c += kSchedThreads / kWave) {
        uint32_t tot;
        wave_excl_scan(h2[c][lane_id()], &tot);
        if (lane_id() == 0) hist[blockIdx.x * kSchedClasses + c] = tot;
    }
}

__global__ __launch_bounds__(kSchedThreads) void sched_scatter_kernel(const uint32_t *len,
                                                                     uint32_t nblk, uint32_t ntile,
                                                                     const uint32_t *hist,
                                                                     uint32_t *order) {
    constexpr uint32_t kScan = 128;  // classes padded to a power of two
    static_assert(kSchedClasses <= kScan && kScan <= kSchedThreads, "one thread per class");
    __shared__ uint32_t tot[kScan], base[kScan], h[kScan], suf[2][kScan];
    const uint32_t t = threadIdx.x;
    if (t < kScan) {
        uint32_t all = 0, before = 0;
        if (t < kSchedClasses) {
            for (uint32_t w0 = 0; w0 < ntile; w0 += 4) {  // four tiles' counts in flight
                uint32_t x[4];
#pragma unroll
                for (uint32_t k = 0; k < 4; k++) x[k] = w0 + k < ntile ? hist[(w0 + k) * kSchedClasses + t] : 0u;
#pragma unroll
                for (uint32_t k = 0; k < 4; k++) {
                    all += x[k];
                    before += w0 + k < blockIdx.x ? x[k] : 0u;
                }
            }
        }
        tot[t] = all;
        base[t] = before;
        h[t] = 0;
        suf[0][t] = all;
    }
    __syncthreads();
    // every block of a larger class comes first: suffix sums over the classes
    // (a log-step scan; a serial sum per class was 124 dependent LDS reads)
    uint32_t sp = 0;
    for (uint32_t d = 1; d < kScan; d <<= 1) {
        if (t < kScan) suf[sp ^ 1][t] = suf[sp][t] + (t + d < kScan ? suf[sp][t + d] : 0u);
        sp ^= 1;
        __syncthreads();
    }
    if (t < kScan) base[t] += suf[sp][t] - tot[t];
    __syncthreads();
    const uint32_t t0 = blockIdx.x * kSchedTile + threadIdx.x;
    uint32_t n[kSchedPer];
#pragma unroll
    for (uint32_t u = 0; u < kSchedPer; u++) {
        const uint32_t i = t0 + u * kSchedThreads;
        n[u] = i < nblk ? len[i] : 0;
    }
#pragma unroll
    for (uint32_t u = 0; u < kSchedPer; u++) {
        const uint32_t i = t0 + u * kSchedThreads;
        if (i < nblk) {
            const uint32_t c = size_class(n[u]);
            order[base[c] + atomicAdd(&h[c], 1u)] = i;
        }
    }
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
//   Steps 2-4 run in sst_tail_kernel, one 256-thread workgroup per file
//   (three launches of a wave per file each took ~4.8 us: 14.6 -> 4.8 us):
//   2. wave 0 chases the index from the first entry the hypothesis failed
//      on (decode_range_v2, exact semantics).
//   3. only when it did fail: the values are located by the index offsets
//      (SSTable.EncodeTo writes value i at Indexes[i].Offset,
//      sstable.go:164-169); value i is verified when it starts where value
//      i-1 ended (value 0 at DataHandle.Offset) and ends where value i+1
//      starts (the last one at the end of the region).  The verified values
//      are exactly the serial chase's.  (Under the hypothesis
//      sst_index_kernel checked them already.)
//   4. wave 0 chases the data region from the first unverified value, then
//      applies GetKeyValuePairs' count rules and writes the per-file
//      lsm_sst_meta.
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
    // words needed for nb bits, without the (nb + 63) overflow (nb near 2^64)
    if (nb / 64 + ((nb & 63) != 0) > (L - 24) / 8) { m.stage = LSM_SST_FILTER; return; }
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
    uint32_t *fail;  // [3f] first unverified index entry, [3f+1] first unverified value,
                     // [3f+2] the same under the stride hypothesis (sst_index_kernel)
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
    // Entry i at io + i S (the stride hypothesis: every key has the first
    // key's length), and in the same pass value i, located by the entry's
    // offset and checked against the next entry's (sst_tail_kernel's step 3
    // rule).  The value checks stand only if the hypothesis holds for the
    // whole index; sst_tail_kernel decides, and otherwise checks the values
    // again from the final offsets.
    const uint64_t S = 12ull + W.k0;
    const uint64_t doff = (uint64_t)W.m.data_off, dl = W.dl;
    const bool whole = (uint64_t)W.spec_cnt * S == W.il && !W.idx_overrun;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < W.spec_cnt;
         i += gridDim.x * blockDim.x) {
        const uint64_t p = W.io + (uint64_t)i * S;
        const bool ok = R.u32(p) == W.k0;
        // the next entry's key length and offset: one round trip with this one's
        const bool has_next = i + 1 < W.spec_cnt;
        const uint32_t k_next = has_next ? R.u32(p + S) : W.k0;
        const uint64_t o_next = has_next ? R.u64(p + S + 4 + W.k0) : 0;
        if (ok) {
            const uint64_t ro = foff + p;
            u32x4 d;
            d.x = (uint32_t)ro;
            d.y = (uint32_t)(ro >> 32);
            d.z = W.k0;
            d.w = 8;
            // nt: the views are read by a later call, not by this one
            // (the f1 line: 141 -> 135 us per call)
            __builtin_nontemporal_store(d, &a.idx_desc[W.base + i]);
            const uint64_t v = R.u64(p + 4 + W.k0);
            a.idx_value[W.base + i] = (int64_t)v;
            if (!W.data_neg && (has_next ? k_next == W.k0 : whole)) {
                const uint64_t pos = v - doff;  // value i, region-relative
                bool bad = dl < 4 || pos > dl - 4 || (i == 0 && pos != 0);
                if (!bad) {
                    const uint32_t vl = R.u32(W.dof + pos);
                    const uint64_t e = pos + 4 + vl;  // where value i ends
                    const uint64_t next = has_next ? o_next - doff : dl;
                    bad = e > dl || e != next;
                    const uint64_t vo = foff + W.dof + pos;
                    u32x4 dd;
                    dd.x = (uint32_t)vo;
                    dd.y = (uint32_t)(vo >> 32);
                    dd.z = 0;
                    dd.w = vl;
                    __builtin_nontemporal_store(dd, &a.data_desc[W.base + i]);
                }
                if (bad) atomicMin(&a.fail[3 * f + 2], i);
            }
        } else {
            atomicMin(&a.fail[3 * f], i);
        }
    }
}

// Steps 2-4 for one file in one workgroup (wave 0 chases, the workgroup
// verifies): a file whose index held the stride hypothesis had its values
// verified by sst_index_kernel and takes one pass of wave 0.
__global__ __launch_bounds__(256) void sst_tail_kernel(SstArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t ring[8 * kChunk / 4 + 4];
    __shared__ uint32_t s_nidx, s_hyp, s_fail;
    __shared__ int32_t s_stage, s_status;
    const uint32_t f = blockIdx.x, t = threadIdx.x;
    SstWork &W = a.work[f];
    const int32_t stage0 = (int32_t)uni((uint32_t)W.m.stage);
    if (t < kWave) {
        // 2. the index
        uint32_t nidx = 0;
        bool hyp = false;
        int32_t st = LSM_OK;
        if (stage0 == 0) {
            const uint32_t spec = uni(W.spec_cnt);
            const uint32_t fl = uni(a.fail[3 * f]);
            const uint32_t i0 = fl < spec ? fl : spec;
            const uint64_t S = 12ull + uni(W.k0), il = uni64(W.il);
            const bool overrun = uni(W.idx_overrun) != 0;
            hyp = i0 == spec && (uint64_t)spec * S == il && !overrun;
            if (hyp) {
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
        }
        if (t == 0) {
            // the index's outcome stays on chip (no re-read of W's fields
            // through the vector cache after a store to them)
            s_stage = st != LSM_OK ? (int32_t)LSM_SST_INDEX : stage0;
            s_status = st != LSM_OK ? st : (int32_t)W.m.status;
            s_nidx = nidx;
            s_hyp = (stage0 == 0 && st == LSM_OK && !hyp && !uni(W.data_neg)) ? 1u : 0u;
            s_fail = hyp ? a.fail[3 * f + 2] : 0xFFFFFFFFu;
        }
    }
    __syncthreads();
    // 3. the values from the final offsets when the index did not hold the
    //    hypothesis (by the whole workgroup)
    if (s_hyp) {
        const uint64_t foff = a.file_off[f];
        ImgReader R;
        R.init(a.img, foff, a.file_len[f]);
        const uint64_t doff = (uint64_t)W.m.data_off, dl = W.dl, base = W.base, dof = W.dof;
        const uint32_t nidx = s_nidx;
        uint32_t mine = 0xFFFFFFFFu;
        for (uint32_t i = t; i < nidx; i += blockDim.x) {
            const uint64_t pos = (uint64_t)a.idx_value[base + i] - doff;  // value i, region-relative
            bool bad = dl < 4 || pos > dl - 4 || (i == 0 && pos != 0);
            if (!bad) {
                const uint32_t v = R.u32(dof + pos);
                const uint64_t e = pos + 4 + v;  // where value i ends
                const uint64_t next = i + 1 < nidx ? (uint64_t)a.idx_value[base + i + 1] - doff : dl;
                bad = e > dl || e != next;
                const uint64_t ro = foff + dof + pos;
                u32x4 d;
                d.x = (uint32_t)ro;
                d.y = (uint32_t)(ro >> 32);
                d.z = 0;
                d.w = v;
                __builtin_nontemporal_store(d, &a.data_desc[base + i]);
            }
            if (bad && i < mine) mine = i;
        }
        if (mine != 0xFFFFFFFFu) atomicMin(&s_fail, mine);
        __syncthreads();
    }
    if (t >= kWave) return;
    // 4. the data region and the file's meta
    int32_t stage = s_stage;
    int32_t status = s_status;
    const uint32_t nidx = s_nidx;
    uint32_t ndata = 0;
    if (stage == LSM_SST_OK) {
        if (uni(W.data_neg)) {
            stage = LSM_SST_DATA;  // seek to a negative offset
        } else {
            const uint32_t fl = uni(s_fail);
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
    if (t == 0) {
        lsm_sst_meta m = W.m;
        m.nidx = nidx;
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
//   wal_seg_lanes_kernel: the segment guesses where its first record starts
//     (the first position from which two records in a row have plausible
//     lengths).  A record is two length-prefixed fields, so a chain started
//     at a value-length field looks just as plausible, one field out of
//     phase, and never meets the true chain: phase 0 starts at the guess g,
//     phase 1 at g + 4 + u32(g) (the record after the value if g was a
//     value length).  Each phase is chased to the first record starting in
//     the next segment, its records written to a scratch area of its own.
//   wal_stitch_kernel: one wave per log walks the segments in order with the
//     true chain position e (0 at the start).  A chain of the segment that
//     starts at e is the serial chase's (same start, same deterministic
//     chain); if neither does, the segment is chased again from e.  The
//     first error ends the log, as it ends Recover.
//   wal_compact_kernel: each segment's records move to their final slots.
// The result equals one serial chase for any input; guesses only decide how
// much is chased twice.
constexpr uint32_t kWalSeg = 16 * 1024;  // 12 and 8 KiB measured slower
constexpr uint32_t kWalSegSlots = kWalSeg / 8 + 1;  // records starting in a segment
// Scratch entry of a record of a segment's chain (wal_seg_lanes_kernel): its
// start less the segment's start (14 bits) and its key length (18 bits;
// kWalKlEsc: re-read from the log).  The value length is the distance to the
// next record's start (or to the chain's exit) less 8 + the key length: 4
// bytes per record and phase instead of a 16-byte descriptor (the scratch
// round trip was 1.9x the replay's algorithmic bytes).
constexpr uint32_t kWalPosBits = 14;
constexpr uint32_t kWalKlEsc = (1u << (32 - kWalPosBits)) - 1;
static_assert(kWalSeg <= (1u << kWalPosBits), "segment offsets fit the scratch entry");
// fin[2q + 1] flags: the chosen phase, and a segment the stitch chased again
// (its records in the scratch as full descriptors)
constexpr uint32_t kWalFinPhase1 = 0x80000000u, kWalFinFull = 0x40000000u, kWalFinCount = 0x3FFFFFFFu;

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

// Lane-parallel segment chase.  WAL records are small
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
    // bytes [x, x+4) and [y, y+4): both from LDS in one round trip when both
    // lie in the copy (the common case), else one at a time
    __device__ __forceinline__ void rd32x2(uint32_t x, uint32_t y, uint32_t &u, uint32_t &v) const {
        const uint32_t ox = h + x - s0, oy = h + y - s0;  // wraps above sz when below s0
        if (ox <= sz - 8 && oy <= sz - 8) {
            const uint32_t a0 = lds[ox >> 2], a1 = lds[(ox >> 2) + 1];
            const uint32_t b0 = lds[oy >> 2], b1 = lds[(oy >> 2) + 1];
            u = funnel(a0, a1, ox);
            v = funnel(b0, b1, oy);
        } else {
            u = rd32(x);
            v = rd32(y);
        }
    }
    // chase() of two chains at once (a lane's two guesses): each step reads
    // both chains' key lengths in one LDS round trip, then both value lengths
    // (the chains are independent; chased one after the other they were two
    // serial chains of dependent reads).  `park` is a position inside the copy
    // for a chain that has stopped.  Same results as two chase() calls.
    __device__ __forceinline__ void chase2(uint32_t pa, uint32_t pb, uint32_t end, uint32_t park,
                                           uint32_t &ca, uint32_t &xa, int32_t &sa, uint32_t &cb,
                                           uint32_t &xb, int32_t &sb) const {
        chase2(pa, pb, end, end, park, ca, xa, sa, cb, xb, sb);
    }
    // the same with an end per chain
    __device__ __forceinline__ void chase2(uint32_t pa, uint32_t pb, uint32_t enda, uint32_t endb,
                                           uint32_t park, uint32_t &ca, uint32_t &xa, int32_t &sa,
                                           uint32_t &cb, uint32_t &xb, int32_t &sb) const {
        ca = cb = 0;
        sa = sb = LSM_OK;
        bool ra = pa < enda && pa < len, rb = pb < endb && pb < len;
        while (ra || rb) {
            // kv.go:77-115 order, as record(): length prefix, key, value length, value
            const uint32_t rma = len - pa, rmb = len - pb;
            const bool ka_ok = ra && rma >= 4, kb_ok = rb && rmb >= 4;
            uint32_t ka, kb;
            rd32x2(ka_ok ? pa : park, kb_ok ? pb : park, ka, kb);
            const bool ka2 = ka_ok && ka <= kKeyCap && rma - 4 >= ka && rma - 4 - ka >= 4;
            const bool kb2 = kb_ok && kb <= kKeyCap && rmb - 4 >= kb && rmb - 4 - kb >= 4;
            uint32_t va, vb;
            rd32x2(ka2 ? pa + 4 + ka : park, kb2 ? pb + 4 + kb : park, va, vb);
            if (ra) {
                int32_t st = LSM_OK;
                if (!ka_ok) st = LSM_ST_TRUNC_LEN_PREFIX;
                else if (ka > kKeyCap) st = LSM_ST_KEY_TOO_LONG;
                else if (rma - 4 < ka) st = LSM_ST_TRUNC_KEY;
                else if (rma - 4 - ka < 4) st = LSM_ST_TRUNC_VLEN;
                else if (va > kValCap) st = LSM_ST_VAL_TOO_LONG;
                else if (rma - 8 - ka < va) st = LSM_ST_TRUNC_VAL;
                if (st != LSM_OK) {
                    sa = st;
                    ra = false;
                } else {
                    ca++;
                    pa += 8 + ka + va;
                    ra = pa < enda && pa < len;
                }
            }
            if (rb) {
                int32_t st = LSM_OK;
                if (!kb_ok) st = LSM_ST_TRUNC_LEN_PREFIX;
                else if (kb > kKeyCap) st = LSM_ST_KEY_TOO_LONG;
                else if (rmb - 4 < kb) st = LSM_ST_TRUNC_KEY;
                else if (rmb - 4 - kb < 4) st = LSM_ST_TRUNC_VLEN;
                else if (vb > kValCap) st = LSM_ST_VAL_TOO_LONG;
                else if (rmb - 8 - kb < vb) st = LSM_ST_TRUNC_VAL;
                if (st != LSM_OK) {
                    sb = st;
                    rb = false;
                } else {
                    cb++;
                    pb += 8 + kb + vb;
                    rb = pb < endb && pb < len;
                }
            }
        }
        xa = pa;
        xb = pb;
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
    // The first plausible start in [ss, se), every position of which lies in
    // the LDS copy (a lane's share of its segment).  A plausible start holds a
    // key length <= 1024, so its u32 has two zero high bytes: positions are
    // screened 16 at a time from five LDS dwords read together, and only the
    // (few) that pass -- in KV logs the length fields -- are tested in full.
    // (Testing every position in full was a serial chain of ~40 dependent
    // LDS round trips per lane.)
    __device__ __forceinline__ uint32_t first_plausible(uint32_t ss, uint32_t se) const {
        const uint32_t ob = h - s0;  // LDS byte offset of log position 0 (mod 2^32)
        for (uint32_t w = (ob + ss) >> 2; 4 * w < ob + se; w += 4) {
            uint32_t d[5];
#pragma unroll
            for (uint32_t t = 0; t < 5; t++) d[t] = lds[w + t];
            uint32_t m = 0;
#pragma unroll
            for (uint32_t j = 0; j < 16; j++) {
                const uint32_t x = funnel(d[j >> 2], d[(j >> 2) + 1], j);
                const uint32_t p = 4 * w + j - ob;
                m |= (uint32_t)(x <= 1024u && p >= ss && p < se) << j;
            }
            while (m) {
                const uint32_t p = 4 * w + (uint32_t)__builtin_ctz(m) - ob;
                if (plausible(p)) return p;
                m &= m - 1;
            }
        }
        return 0xFFFFFFFFu;
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
__global__ __launch_bounds__(64) void wal_seg_lanes_kernel(WalArgs a) {
    constexpr uint32_t STAGE = kWalStage;
    __shared__ __attribute__((aligned(16))) uint32_t stage[STAGE / 4 + 4];
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
    L.s0 = (L.h + start) & ~15u;
    L.sz = STAGE;
    L.lds = stage;
    {
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
        e0 = L.first_plausible(ss, se);
        if (e0 != 0xFFFFFFFFu && (uint64_t)e0 + 4 <= len) {
            const uint32_t v = L.rd32(e0);
            if ((uint64_t)e0 + 4 + v <= len) e1 = e0 + 4 + v;
        }
    }
    // A guess at or past the share's end is a chain with no records that
    // passes its position through (exit = the guess); chase() returns exactly
    // that.  Leaving its exit unset once made a share holding only a value
    // field report exit 0 when the previous chain ended on that guess.
    {
        // both guesses' chains at once; a missing guess is a stopped chain
        // (its count, exit and status keep their initial values)
        uint32_t ca, xa, cb, xb;
        int32_t sa, sb;
        L.chase2(e0 != 0xFFFFFFFFu ? e0 : se, e1 != 0xFFFFFFFFu ? e1 : se, se, start, ca, xa, sa, cb,
                 xb, sb);
        if (e0 != 0xFFFFFFFFu) { c0 = ca; x0 = xa; st0 = sa; }
        if (e1 != 0xFFFFFFFFu) { c1 = cb; x1 = xb; st1 = sb; }
    }
    // The share holding each phase's entry is chased exactly from the entry
    // (the fast stitch below), both phases together.
    uint32_t kc[2], cc[2], xc[2];
    int32_t sc[2];
    {
        const uint32_t live1 = s > 0 && g1 < E;  // phase 1 exists (g < E always)
        kc[0] = (g - start) / W;
        kc[1] = live1 ? (g1 - start) / W : 0;
        const uint32_t se0 = uni(__builtin_amdgcn_readlane(se, kc[0]));
        const uint32_t se1 = uni(__builtin_amdgcn_readlane(se, kc[1]));
        L.chase2(g, live1 ? g1 : se1, se0, se1, start, cc[0], xc[0], sc[0], cc[1], xc[1], sc[1]);
#pragma unroll
        for (uint32_t i = 0; i < 2; i++) {
            cc[i] = uni(cc[i]);
            xc[i] = uni(xc[i]);
            sc[i] = (int32_t)uni((uint32_t)sc[i]);
        }
    }
    // 2. per phase: stitch from the entry (each lane's accepted chain)
    uint32_t wpre[2] = {0, 0}, wentry[2] = {0, 0}, wcnt[2] = {0, 0};
#pragma unroll
    for (uint32_t ph = 0; ph < 2; ph++) {
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
            const uint32_t k = kc[ph];
            const uint32_t last = (E - 1 - start) / W < kWave - 1 ? (E - 1 - start) / W : kWave - 1;
            const uint32_t ck = cc[ph], xk = xc[ph];
            const int32_t stk = sc[ph];
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
        wpre[ph] = wave_excl_scan(acc_cnt, &tot);
        wentry[ph] = acc_entry;
        wcnt[ph] = acc_cnt;
        if (lane == 0) a.seg[q] = WalSeg{gp, e, total, status};
    }
    // 3. both phases' accepted chains walked together, a 4-byte scratch entry
    //    per record: each step reads both key lengths in one LDS round trip,
    //    then both value lengths (walked one phase after the other they were
    //    two serial chains: 1,117 -> 1,167 GiB/s, A/B)
    {
        uint32_t *dst0 = reinterpret_cast<uint32_t *>(a.scratch + q0 * kWalSegSlots) + wpre[0];
        uint32_t *dst1 = reinterpret_cast<uint32_t *>(a.scratch + (q0 + 1) * kWalSegSlots) + wpre[1];
        uint32_t pa = wentry[0], pb = wentry[1];
        const uint32_t n = wcnt[0] > wcnt[1] ? wcnt[0] : wcnt[1];
        for (uint32_t i = 0; i < n; i++) {
            const bool ra = i < wcnt[0], rb = i < wcnt[1];
            uint32_t ka, kb, va, vb;
            L.rd32x2(ra ? pa : start, rb ? pb : start, ka, kb);
            L.rd32x2(ra ? pa + 4 + ka : start, rb ? pb + 4 + kb : start, va, vb);
            if (ra) {
                dst0[i] = (pa - start) | (ka < kWalKlEsc ? ka : kWalKlEsc) << kWalPosBits;
                pa += 8 + ka + va;
            }
            if (rb) {
                dst1[i] = (pb - start) | (kb < kWalKlEsc ? kb : kWalKlEsc) << kWalPosBits;
                pb += 8 + kb + vb;
            }
        }
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
                f_cnt = nr | (take && ch == 1 ? kWalFinPhase1 : 0u);
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
                cnt = nr | (ph == 1 ? kWalFinPhase1 : ph == 2 ? kWalFinFull : 0u);
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
    const uint32_t cnt = cf & kWalFinCount;
    if (cnt == 0) return;
    uint64_t base, cap;
    wal_slots(a, w, base, cap);
    u32x4 *dst = reinterpret_cast<u32x4 *>(a.out.desc);
    const uint32_t ph = cf >> 31;
    if (cf & kWalFinFull) {  // chased again by the stitch: full descriptors
        const u32x4 *src = a.scratch + q * 2 * kWalSegSlots;
        for (uint32_t j = threadIdx.x; j < cnt; j += blockDim.x)
            if ((uint64_t)pre + j < cap)  // nt: written once (A/B: 997 -> 1,017 GiB/s)
                __builtin_nontemporal_store(src[j], &dst[base + pre + j]);
        return;
    }
    // packed entries: record j ends where record j + 1 starts (the chain's
    // exit after the last), so its value length is that distance less 8 +
    // its key length
    const uint32_t *src = reinterpret_cast<const uint32_t *>(a.scratch + (q * 2 + ph) * kWalSegSlots);
    const uint64_t start = (uint64_t)a.wal_off[w] + (uint64_t)s * kWalSeg;
    const uint32_t rel_exit = a.seg[q * 2 + ph].exit - s * kWalSeg;
    for (uint32_t j = threadIdx.x; j < cnt; j += blockDim.x) {
        if ((uint64_t)pre + j >= cap) continue;
        const uint32_t e = src[j];
        const uint32_t p = e & ((1u << kWalPosBits) - 1);
        const uint32_t pn = j + 1 < cnt ? (src[j + 1] & ((1u << kWalPosBits) - 1)) : rel_exit;
        uint32_t kl = e >> kWalPosBits;
        if (kl == kWalKlEsc) {  // a key of 2^18 bytes or more: its length from the log
            const uint8_t *kp = a.wal + start + p;
            kl = (uint32_t)kp[0] | (uint32_t)kp[1] << 8 | (uint32_t)kp[2] << 16 | (uint32_t)kp[3] << 24;
        }
        const uint64_t ro = start + p;
        __builtin_nontemporal_store(u32x4{(uint32_t)ro, (uint32_t)(ro >> 32), kl, pn - p - 8 - kl},
                                    &dst[base + pre + j]);
    }
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
    a.order = nullptr;
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (grammar) {
    case LSM_GRAMMAR_V: return arena ? launch_decode<LSM_GRAMMAR_V, true>(a, s)
                                     : launch_decode<LSM_GRAMMAR_V, false>(a, s);
    case LSM_GRAMMAR_KV: return arena ? launch_decode<LSM_GRAMMAR_KV, true>(a, s)
                                      : launch_decode<LSM_GRAMMAR_KV, false>(a, s);
    default: return arena ? launch_decode<LSM_GRAMMAR_IDX, true>(a, s)
                          : launch_decode<LSM_GRAMMAR_IDX, false>(a, s);
    }
}

// A caller that knows its blocks are large (max_blk_len > 32 KiB: 64 KiB data
// blocks, whole index regions) gets a 16 KiB ring: twice the bytes in flight
// per wave (6,400 x 64 KiB blocks: 89.5 against 92.6 us).  The hint only
// picks the ring; any block length decodes correctly either way.
extern "C" int lsm_decode_blocks_hinted(lsm_ctx *ctx, int grammar, const uint8_t *d_in,
                                        const uint64_t *d_blk_off, const uint32_t *d_blk_len,
                                        uint32_t nblk, uint32_t max_blk_len,
                                        const lsm_decode_out *out, void *stream) {
    if (max_blk_len <= 32 * 1024)
        return lsm_decode_blocks(ctx, grammar, d_in, d_blk_off, d_blk_len, nblk, out, stream);
    if (!ctx || !out) return LSM_EINVAL;
    if (nblk == 0) return 0;
    if (!d_in || !d_blk_off || !d_blk_len || !out->desc || !out->nrec || !out->status)
        return LSM_EINVAL;
    if (grammar < LSM_GRAMMAR_V || grammar > LSM_GRAMMAR_IDX) return LSM_EINVAL;
    const bool arena = out->key_arena || out->val_arena;
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
    a.order = nullptr;
    hipStream_t s = static_cast<hipStream_t>(stream);
    constexpr uint32_t R = 2 * kRingChunks;
    switch (grammar) {
    case LSM_GRAMMAR_V: return arena ? launch_decode<LSM_GRAMMAR_V, true, R>(a, s)
                                     : launch_decode<LSM_GRAMMAR_V, false, R>(a, s);
    case LSM_GRAMMAR_KV: return arena ? launch_decode<LSM_GRAMMAR_KV, true, R>(a, s)
                                      : launch_decode<LSM_GRAMMAR_KV, false, R>(a, s);
    default: return arena ? launch_decode<LSM_GRAMMAR_IDX, true, R>(a, s)
                          : launch_decode<LSM_GRAMMAR_IDX, false, R>(a, s);
    }
}

extern "C" size_t lsm_decode_schedule_workspace_bytes(uint32_t nblk) {
    const uint64_t ntile = ((uint64_t)nblk + kSchedTile - 1) / kSchedTile;
    return 4ull * kSchedClasses * ntile + 4ull * nblk + 16;
}

extern "C" int lsm_decode_blocks_scheduled(lsm_ctx *ctx, int grammar, const uint8_t *d_in,
                                           const uint64_t *d_blk_off, const uint32_t *d_blk_len,
                                           uint32_t nblk, const lsm_decode_out *out,
                                           void *d_workspace, size_t ws_bytes, void *stream) {
    if (!ctx || !out) return LSM_EINVAL;
    if (nblk == 0) return 0;
    if (!d_in || !d_blk_off || !d_blk_len || !out->desc || !out->nrec || !out->status)
        return LSM_EINVAL;
    if (grammar < LSM_GRAMMAR_V || grammar > LSM_GRAMMAR_IDX) return LSM_EINVAL;
    if (!d_workspace || ws_bytes < lsm_decode_schedule_workspace_bytes(nblk)) return LSM_ESPACE;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint32_t ntile = (nblk + kSchedTile - 1) / kSchedTile;
    uint32_t *order = static_cast<uint32_t *>(d_workspace);
    uint32_t *hist = order + nblk;
    hipLaunchKernelGGL(sched_hist_kernel, dim3(ntile), dim3(kSchedThreads), 0, s, d_blk_len, nblk,
                       hist);
    hipLaunchKernelGGL(sched_scatter_kernel, dim3(ntile), dim3(kSchedThreads), 0, s, d_blk_len, nblk,
                       ntile, hist, order);
    LSM_HIP_CHECK(hipGetLastError());
    const bool arena = out->key_arena || out->val_arena;
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
    a.order = order;
    // mixed sizes: a 2 KiB ring, the most waves per CU (config 5: 201 us, 4 KiB
    // 215 us, 8 KiB 231 us; the 8 KiB ring streams uniform 64 KiB blocks
    // fastest: 92 against 100 us with 4 KiB).  Quarter-octave classes measured
    // the same as sixteenth-octave ones.
    constexpr uint32_t R = kRingChunks / 4;
    switch (grammar) {
    case LSM_GRAMMAR_V: return arena ? launch_decode<LSM_GRAMMAR_V, true, R>(a, s)
                                     : launch_decode<LSM_GRAMMAR_V, false, R>(a, s);
    case LSM_GRAMMAR_KV: return arena ? launch_decode<LSM_GRAMMAR_KV, true, R>(a, s)
                                      : launch_decode<LSM_GRAMMAR_KV, false, R>(a, s);
    default: return arena ? launch_decode<LSM_GRAMMAR_IDX, true, R>(a, s)
                          : launch_decode<LSM_GRAMMAR_IDX, false, R>(a, s);
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
    hipLaunchKernelGGL(wal_seg_lanes_kernel, dim3(a.segs, nwal), dim3(kWave), 0, s, a);
    hipLaunchKernelGGL(wal_stitch_kernel, dim3(nwal), dim3(kWave), 0, s, a);
    hipLaunchKernelGGL(wal_compact_kernel, dim3(a.segs, nwal), dim3(256), 0, s, a);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}

extern "C" size_t lsm_decode_sst_workspace_bytes(uint32_t nfile) {
    return (size_t)nfile * (sizeof(SstWork) + 12) + 16;
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
    LSM_HIP_CHECK(hipMemsetAsync(a.fail, 0xFF, (size_t)nfile * 12, s));
    // parallel passes: ~kSstWgs workgroups over the batch, at most 64 per file (about one
    // index entry per thread for a 2 MiB file; 2,048 / 8,192 / 16,384 measured 126.4 / 120.0 /
    // 111.6 us for 208 files, A/B)
    constexpr uint32_t kSstWgs = 16384;
    uint32_t g = (kSstWgs + nfile - 1) / nfile;
    if (g > 64) g = 64;
    if (g == 0) g = 1;
    hipLaunchKernelGGL(sst_index_kernel, dim3(g, nfile), dim3(256), 0, s, a);
    hipLaunchKernelGGL(sst_tail_kernel, dim3(nfile), dim3(256), 0, s, a);
    LSM_HIP_CHECK(hipGetLastError());
    return 0;
}

