/*
 * lsm_oracle.c — CPU restatement of the go-lsm block-codec path.
 * TEST INFRASTRUCTURE ONLY (see lsm_oracle.h).  Citations are
 * path:line in xmh1011/go-lsm @ 2025-08-24.
 */
#include "lsm_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ---- little/big-endian helpers (encoding/binary) ---------------------- */

static inline uint32_t ld_u32le(const uint8_t *p) {
    return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}
static inline uint64_t ld_u64le(const uint8_t *p) {
    return (uint64_t)ld_u32le(p) | (uint64_t)ld_u32le(p + 4) << 32;
}
static inline uint64_t ld_u64be(const uint8_t *p) {
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v = v << 8 | p[i];
    return v;
}
static inline void st_u32le(uint8_t *p, uint32_t v) {
    for (int i = 0; i < 4; i++) p[i] = (uint8_t)(v >> (8 * i));
}
static inline void st_u64le(uint8_t *p, uint64_t v) {
    for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (8 * i));
}
static inline void st_u64be(uint8_t *p, uint64_t v) {
    for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (8 * (7 - i)));
}

#define KEY_CAP (1u << 20) /* kv.go:84  */
#define VAL_CAP (1u << 30) /* kv.go:102 */

/* ---- record decode ---------------------------------------------------- */

int ora_decode_block(int grammar, const uint8_t *base, uint64_t blk_off, uint64_t blk_len,
                     ora_desc *desc, int64_t *idx_val, uint64_t cap, uint32_t *nrec) {
    const uint8_t *b = base + blk_off;
    const uint64_t n = blk_len;
    uint64_t pos = 0;
    uint64_t cnt = 0;
    int st = ORA_OK;

    if (grammar == ORA_GRAMMAR_V) {
        /* data.go:58-76: loop { binary.Read u32; EOF -> stop; short -> error;
         * make(valLen); ReadFull; append }.  The block is the LimitReader. */
        for (;;) {
            uint64_t rem = n - pos;
            if (rem == 0) break;                                 /* io.EOF, :62-63  */
            if (rem < 4) { st = ORA_TRUNC_LEN_PREFIX; break; }   /* :65-66          */
            uint32_t vlen = ld_u32le(b + pos);
            if (rem - 4 < vlen) { st = ORA_TRUNC_VAL; break; }   /* :71-73          */
            if (cnt >= cap) { st = ORA_CAPACITY; break; }
            desc[cnt].rec_off = blk_off + pos;
            desc[cnt].key_len = 0;
            desc[cnt].val_len = vlen;
            cnt++;
            pos += 4 + (uint64_t)vlen;
        }
    } else if (grammar == ORA_GRAMMAR_KV) {
        /* wal.go:107 `for buf.Len() > 0` around KeyValuePair.DecodeFrom kv.go:77-115 */
        while (pos < n) {
            uint64_t rem = n - pos;
            if (rem < 4) { st = ORA_TRUNC_LEN_PREFIX; break; }   /* kv.go:80-82   */
            uint32_t klen = ld_u32le(b + pos);
            if (klen > KEY_CAP) { st = ORA_KEY_TOO_LONG; break; } /* kv.go:84-86  */
            if (rem - 4 < klen) { st = ORA_TRUNC_KEY; break; }    /* kv.go:90-92  */
            uint64_t vp = pos + 4 + klen;
            uint64_t rem2 = n - vp;
            if (rem2 < 4) { st = ORA_TRUNC_VLEN; break; }         /* kv.go:98-100 */
            uint32_t vlen = ld_u32le(b + vp);
            if (vlen > VAL_CAP) { st = ORA_VAL_TOO_LONG; break; } /* kv.go:102-104 */
            if (rem2 - 4 < vlen) { st = ORA_TRUNC_VAL; break; }   /* kv.go:108-110 */
            if (cnt >= cap) { st = ORA_CAPACITY; break; }
            desc[cnt].rec_off = blk_off + pos;
            desc[cnt].key_len = klen;
            desc[cnt].val_len = vlen;
            cnt++;
            pos = vp + 4 + vlen;
        }
    } else if (grammar == ORA_GRAMMAR_IDX) {
        /* index.go:70-98: while totalRead < size { Key.DecodeFrom; read i64;
         * totalRead += 4+klen+8; if totalRead > size -> error }.  Bytes past
         * the block are treated as present (the .sst footer follows the
         * index), so any entry crossing the limit is the overrun error. */
        while (pos < n) {
            uint64_t rem = n - pos;
            if (rem < 4) { st = ORA_IDX_OVERRUN; break; }
            uint32_t klen = ld_u32le(b + pos);
            if (rem < 12 + (uint64_t)klen) { st = ORA_IDX_OVERRUN; break; }
            if (cnt >= cap) { st = ORA_CAPACITY; break; }
            desc[cnt].rec_off = blk_off + pos;
            desc[cnt].key_len = klen;
            desc[cnt].val_len = 8;
            if (idx_val) idx_val[cnt] = (int64_t)ld_u64le(b + pos + 4 + klen);
            cnt++;
            pos += 12 + (uint64_t)klen;
        }
    }
    *nrec = (uint32_t)cnt;
    return st;
}

uint64_t ora_materialize(int grammar, const uint8_t *base, const ora_desc *desc, uint64_t n,
                         uint8_t *key_arena, uint8_t *val_arena, uint64_t *val_bytes) {
    uint64_t kb = 0, vb = 0;
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t *r = base + desc[i].rec_off;
        uint32_t kl = desc[i].key_len, vl = desc[i].val_len;
        if (grammar == ORA_GRAMMAR_V) {
            memcpy(val_arena + vb, r + 4, vl);
            vb += vl;
        } else if (grammar == ORA_GRAMMAR_KV) {
            memcpy(key_arena + kb, r + 4, kl);
            kb += kl;
            memcpy(val_arena + vb, r + 8 + kl, vl);
            vb += vl;
        } else {
            memcpy(key_arena + kb, r + 4, kl);
            kb += kl;
        }
    }
    if (val_bytes) *val_bytes = vb;
    return kb;
}

/* ---- record encode ---------------------------------------------------- */

uint64_t ora_encoded_size(int grammar, const uint64_t *koff, const uint64_t *voff, uint64_t r0,
                          uint64_t r1) {
    uint64_t n = r1 - r0;
    if (grammar == ORA_GRAMMAR_V) return 4 * n + (voff[r1] - voff[r0]);
    if (grammar == ORA_GRAMMAR_KV) return 8 * n + (koff[r1] - koff[r0]) + (voff[r1] - voff[r0]);
    return 12 * n + (koff[r1] - koff[r0]);
}

uint64_t ora_encode_records(int grammar, const uint8_t *keys, const uint64_t *koff,
                            const uint8_t *vals, const uint64_t *voff, uint64_t r0, uint64_t r1,
                            const int64_t *idx_off, uint8_t *out) {
    uint64_t w = 0;
    for (uint64_t i = r0; i < r1; i++) {
        if (grammar == ORA_GRAMMAR_KV || grammar == ORA_GRAMMAR_IDX) {
            uint32_t kl = (uint32_t)(koff[i + 1] - koff[i]); /* uint32(len(key)) kv.go:48 */
            st_u32le(out + w, kl);
            memcpy(out + w + 4, keys + koff[i], kl);
            w += 4 + (uint64_t)kl;
        }
        if (grammar == ORA_GRAMMAR_KV || grammar == ORA_GRAMMAR_V) {
            uint32_t vl = (uint32_t)(voff[i + 1] - voff[i]);
            st_u32le(out + w, vl);
            memcpy(out + w + 4, vals + voff[i], vl);
            w += 4 + (uint64_t)vl;
        } else {
            st_u64le(out + w, (uint64_t)idx_off[i - r0]); /* index.go:37 */
            w += 8;
        }
    }
    return w;
}

/* ---- MurmurHash3 restatement of digest128 (murmur.go) ----------------- */

#define MC1 0x87c37b91114253d5ULL /* murmur.go:52 */
#define MC2 0x4cf5ad432745937fULL /* murmur.go:53 */

static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

static inline uint64_t fmix(uint64_t k) { /* murmur.go:223-230 */
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}

typedef struct { uint64_t h1, h2; } digest;

static void mix_words(digest *d, uint64_t k1, uint64_t k2) { /* bmixWords murmur.go:74-95 */
    uint64_t h1 = d->h1, h2 = d->h2;
    k1 *= MC1; k1 = rotl64(k1, 31); k1 *= MC2; h1 ^= k1;
    h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
    k2 *= MC2; k2 = rotl64(k2, 33); k2 *= MC1; h2 ^= k2;
    h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
    d->h1 = h1; d->h2 = h2;
}

/* sum128 murmur.go:104-221: fold a tail of tl (<16) bytes, then finalize
 * with the total length.  The Go padTail switch ORs a virtual 0x01 byte at
 * tail position len(tail); here the caller passes that byte in `tail`. */
static void finish(const digest *d, uint64_t length, const uint8_t *tail, unsigned tl,
                   uint64_t *o1, uint64_t *o2) {
    uint64_t h1 = d->h1, h2 = d->h2, k1 = 0, k2 = 0;
    for (unsigned i = 8; i < tl; i++) k2 ^= (uint64_t)tail[i] << (8 * (i - 8));
    if (tl > 8) { k2 *= MC2; k2 = rotl64(k2, 33); k2 *= MC1; h2 ^= k2; }
    for (unsigned i = 0; i < tl && i < 8; i++) k1 ^= (uint64_t)tail[i] << (8 * i);
    if (tl > 0) { k1 *= MC1; k1 = rotl64(k1, 31); k1 *= MC2; h1 ^= k1; }
    h1 ^= length; h2 ^= length;
    h1 += h2; h2 += h1;
    h1 = fmix(h1); h2 = fmix(h2);
    h1 += h2; h2 += h1;
    *o1 = h1; *o2 = h2;
}

void ora_sum256(const uint8_t *data, uint64_t len, uint64_t h[4]) { /* murmur.go:245-275 */
    digest d = {0, 0};
    uint64_t nb = len / 16;
    for (uint64_t i = 0; i < nb; i++) mix_words(&d, ld_u64le(data + 16 * i), ld_u64le(data + 16 * i + 8));
    unsigned tl = (unsigned)(len % 16);
    const uint8_t *tail = data + len - tl;
    finish(&d, len, tail, tl, &h[0], &h[1]);
    uint8_t t2[16];
    memcpy(t2, tail, tl);
    t2[tl] = 1; /* virtually append 0x01 (murmur.go:251-270) */
    if (tl + 1 == 16) {
        mix_words(&d, ld_u64le(t2), ld_u64le(t2 + 8));
        finish(&d, len + 1, t2, 0, &h[2], &h[3]);
    } else {
        finish(&d, len + 1, t2, tl + 1, &h[2], &h[3]);
    }
}

/* ---- bloom (bloom.go) -------------------------------------------------- */

uint64_t ora_location(const uint64_t h[4], uint64_t i) { /* bloom.go:133-136 */
    return h[i % 2] + i * h[2 + (((i + (i % 2)) % 4) / 2)];
}

void ora_bloom_add(uint64_t *words, uint64_t m, uint64_t k, const uint8_t *key, uint64_t len) {
    uint64_t h[4];
    uint64_t am = m ? m : 1, hk = k ? k : 1; /* NewBloomFilter max(1,..) bloom.go:95-101 */
    ora_sum256(key, len, h);
    for (uint64_t i = 0; i < hk; i++) {
        uint64_t p = ora_location(h, i) % am; /* bloom.go:139-141 */
        words[p >> 6] |= 1ULL << (p & 63);    /* bitset.Set         */
    }
}

int ora_bloom_test(const uint64_t *words, uint64_t m, uint64_t k, const uint8_t *key,
                   uint64_t len) {
    uint64_t h[4];
    uint64_t am = m ? m : 1, hk = k ? k : 1;
    ora_sum256(key, len, h);
    for (uint64_t i = 0; i < hk; i++) {
        uint64_t p = ora_location(h, i) % am;
        if (!(words[p >> 6] >> (p & 63) & 1)) return 0;
    }
    return 1;
}

int ora_filter_test(const uint64_t *words, uint64_t nbits, uint64_t m, uint64_t k,
                    const uint8_t *key, uint64_t len) {
    uint64_t h[4];
    ora_sum256(key, len, h);                       /* baseHashes, bloom.go:372 */
    for (uint64_t i = 0; i < k; i++) {             /* bloom.go:373, no max(1,k) */
        if (m == 0) return -1;                     /* location(): % 0 panics    */
        uint64_t p = ora_location(h, i) % m;       /* bloom.go:139-141          */
        if (p >= nbits) return 0;                  /* bitset.Test past length   */
        if (!(words[p >> 6] >> (p & 63) & 1)) return 0;
    }
    return 1;
}

void ora_estimate_parameters(uint64_t n, double p, uint64_t *m, uint64_t *k) {
    double ln2 = log(2.0);
    *m = (uint64_t)ceil(-1.0 * (double)n * log(p) / pow(ln2, 2));
    *k = (uint64_t)ceil(ln2 * (double)*m / (double)n);
}

uint64_t ora_filter_block_size(uint64_t m) { return 8 + 24 + 8 * ((m + 63) / 64); }

uint64_t ora_filter_encode(const uint64_t *words, uint64_t m, uint64_t k, uint8_t *out) {
    uint64_t nw = (m + 63) / 64;
    st_u64le(out, 24 + 8 * nw);        /* EncodeTo length prefix, bloom.go:478 */
    st_u64be(out + 8, m ? m : 1);       /* WriteTo arraySize, bloom.go:240     */
    st_u64be(out + 16, k ? k : 1);      /* WriteTo hashNum,  bloom.go:244      */
    st_u64be(out + 24, m);              /* bitset length                        */
    for (uint64_t i = 0; i < nw; i++) st_u64be(out + 32 + 8 * i, words[i]);
    return 32 + 8 * nw;
}

int ora_filter_decode(const uint8_t *in, uint64_t n, uint64_t *m, uint64_t *k, uint64_t *nbits,
                      uint64_t *words, uint64_t words_cap, uint64_t *consumed) {
    if (n < 8) return -1;                       /* "decode filter length"        */
    uint64_t L = ld_u64le(in);
    if (L > n - 8) return -2;                   /* "decode filter data"          */
    const uint8_t *p = in + 8;
    if (L < 24) return -3;                      /* ReadFrom m/k/length short     */
    *m = ld_u64be(p);
    *k = ld_u64be(p + 8);
    *nbits = ld_u64be(p + 16);
    /* words stored for nbits bits, without the (nbits + 63) overflow */
    uint64_t nw = *nbits / 64 + ((*nbits & 63) != 0);
    if (nw > (L - 24) / 8) return -4;           /* bitset.ReadFrom words short   */
    if (words) {
        if (nw > words_cap) return -5;
        for (uint64_t i = 0; i < nw; i++) words[i] = ld_u64be(p + 24 + 8 * i);
    }
    *consumed = 8 + L;
    return 0;
}

/* ---- .sst -------------------------------------------------------------- */

uint64_t ora_segment_files(const uint64_t *koff, const uint64_t *voff, uint64_t n,
                           uint64_t threshold, uint64_t *starts) {
    uint64_t nf = 0, size = 0, start = 0;
    for (uint64_t i = 0; i < n; i++) {
        size += 4 + (koff[i + 1] - koff[i]) + 4 + (voff[i + 1] - voff[i]) + 8; /* kv.go:118-121 */
        if (threshold && size >= threshold) {                                    /* builder.go:40-42 */
            starts[nf++] = start;
            start = i + 1;
            size = 0;
        }
    }
    if (size > 0) starts[nf++] = start; /* merge.go:120-123 */
    starts[nf] = n;
    return nf;
}

static uint64_t header_size(const uint64_t *koff, uint64_t r0, uint64_t r1) {
    if (r1 <= r0) return 8;
    return 8 + (koff[r0 + 1] - koff[r0]) + (koff[r1] - koff[r1 - 1]);
}

uint64_t ora_sst_image_size(const uint64_t *koff, const uint64_t *voff, uint64_t r0, uint64_t r1,
                            uint64_t m) {
    return header_size(koff, r0, r1) + ora_filter_block_size(m) +
           ora_encoded_size(ORA_GRAMMAR_V, koff, voff, r0, r1) +
           ora_encoded_size(ORA_GRAMMAR_IDX, koff, voff, r0, r1) + 32;
}

uint64_t ora_build_sst(const uint8_t *keys, const uint64_t *koff, const uint8_t *vals,
                       const uint64_t *voff, uint64_t r0, uint64_t r1, uint64_t m, uint64_t k,
                       uint8_t *out, int64_t footer_out[4]) {
    uint64_t w = 0;
    /* Header (builder.go:45-53 Finalize; header.go:25-37 EncodeTo) */
    if (r1 > r0) {
        uint32_t l0 = (uint32_t)(koff[r0 + 1] - koff[r0]);
        uint32_t l1 = (uint32_t)(koff[r1] - koff[r1 - 1]);
        st_u32le(out, l0); memcpy(out + 4, keys + koff[r0], l0); w = 4 + l0;
        st_u32le(out + w, l1); memcpy(out + w + 4, keys + koff[r1 - 1], l1); w += 4 + l1;
    } else {
        st_u32le(out, 0); st_u32le(out + 4, 0); w = 8;
    }
    /* Filter (SSTable.Add -> Filter.Add, sstable.go:322-326; EncodeTo bloom.go:472) */
    uint64_t nw = (m + 63) / 64;
    uint64_t *words = (uint64_t *)calloc(nw ? nw : 1, 8);
    for (uint64_t i = r0; i < r1; i++) ora_bloom_add(words, m, k, keys + koff[i], koff[i + 1] - koff[i]);
    w += ora_filter_encode(words, m, k, out + w);
    free(words);
    /* Data region: sstable.go:159-175, offsets by exclusive prefix sum */
    int64_t data_off = (int64_t)w;
    uint64_t n = r1 - r0;
    int64_t *ioff = (int64_t *)malloc((n ? n : 1) * sizeof(int64_t));
    uint64_t cur = w;
    for (uint64_t i = r0; i < r1; i++) {
        ioff[i - r0] = (int64_t)cur;
        cur += 4 + (voff[i + 1] - voff[i]);
    }
    w += ora_encode_records(ORA_GRAMMAR_V, keys, koff, vals, voff, r0, r1, NULL, out + w);
    int64_t data_size = (int64_t)w - data_off;
    /* Index region: sstable.go:178-186 */
    int64_t idx_off = (int64_t)w;
    w += ora_encode_records(ORA_GRAMMAR_IDX, keys, koff, vals, voff, r0, r1, ioff, out + w);
    int64_t idx_size = (int64_t)w - idx_off;
    free(ioff);
    /* Footer footer.go:43-55 */
    st_u64le(out + w, (uint64_t)data_off);
    st_u64le(out + w + 8, (uint64_t)data_size);
    st_u64le(out + w + 16, (uint64_t)idx_off);
    st_u64le(out + w + 24, (uint64_t)idx_size);
    w += 32;
    if (footer_out) {
        footer_out[0] = data_off; footer_out[1] = data_size;
        footer_out[2] = idx_off; footer_out[3] = idx_size;
    }
    return w;
}

int ora_sst_decode(const uint8_t *file, uint64_t n, ora_sst_meta *meta, ora_desc *idx_desc,
                   int64_t *idx_val, uint64_t idx_cap, ora_desc *data_desc, uint64_t data_cap) {
    memset(meta, 0, sizeof(*meta));
    uint64_t pos = 0;
    /* Header.DecodeFrom header.go:40-52 (Key.DecodeFrom kv.go:124-139, no cap) */
    for (int j = 0; j < 2; j++) {
        if (n - pos < 4) { meta->stage = 1; return 1; }
        uint32_t kl = ld_u32le(file + pos);
        if (n - pos - 4 < kl) { meta->stage = 1; return 1; }
        if (j == 0) { meta->min_key_off = pos + 4; meta->min_key_len = kl; }
        else { meta->max_key_off = pos + 4; meta->max_key_len = kl; }
        pos += 4 + (uint64_t)kl;
    }
    /* Filter.DecodeFrom bloom.go:453-469 */
    uint64_t used = 0;
    if (ora_filter_decode(file + pos, n - pos, &meta->filter_m, &meta->filter_k,
                          &meta->filter_nbits, NULL, 0, &used) != 0) {
        meta->stage = 2; return 2;
    }
    meta->filter_words_off = pos + 8 + 24;
    /* DecodeFooterFrom sstable.go:195-212 */
    if (n < 32) { meta->stage = 3; return 3; }
    const uint8_t *f = file + n - 32;
    meta->data_off = (int64_t)ld_u64le(f);
    meta->data_size = (int64_t)ld_u64le(f + 8);
    meta->idx_off = (int64_t)ld_u64le(f + 16);
    meta->idx_size = (int64_t)ld_u64le(f + 24);
    /* IndexBlock.DecodeFrom(file@idx_off, idx_size) sstable.go:116-125, index.go:61-101 */
    if (meta->idx_off < 0) { meta->stage = 4; return 4; }
    if (meta->idx_size < 0) { meta->stage = 4; return 4; } /* index.go:65-68 */
    uint64_t io = (uint64_t)meta->idx_off;
    uint64_t avail = io <= n ? n - io : 0;
    uint64_t il = (uint64_t)meta->idx_size < avail ? (uint64_t)meta->idx_size : avail;
    if ((uint64_t)meta->idx_size > avail) {
        /* the stream ends before the limit: whatever entries fit, then a read error */
        uint32_t c = 0;
        ora_decode_block(ORA_GRAMMAR_IDX, file, io, il, idx_desc, idx_val, idx_cap, &c);
        meta->nidx = c; meta->status = ORA_IDX_OVERRUN; meta->stage = 4; return 4;
    }
    int st = ora_decode_block(ORA_GRAMMAR_IDX, file, io, il, idx_desc, idx_val, idx_cap, &meta->nidx);
    if (st) { meta->status = st; meta->stage = 4; return 4; }
    /* DecodeDataBlock sstable.go:214-225 -> DataBlock.DecodeFrom(file, size):
     * size > 0 -> LimitReader, else unlimited to EOF (data.go:51-54). */
    if (meta->data_off < 0) { meta->stage = 5; return 5; }
    uint64_t dof = (uint64_t)meta->data_off;
    uint64_t davail = dof <= n ? n - dof : 0;
    uint64_t dl = (meta->data_size > 0 && (uint64_t)meta->data_size < davail) ? (uint64_t)meta->data_size : davail;
    st = ora_decode_block(ORA_GRAMMAR_V, file, dof, dl, data_desc, NULL, data_cap, &meta->ndata);
    if (st) { meta->status = st; meta->stage = 5; return 5; }
    /* GetKeyValuePairs sstable.go:248-268 */
    if (meta->ndata == 0 || meta->nidx == 0) return 0;
    if (meta->ndata != meta->nidx) { meta->stage = 6; return 6; }
    return 0;
}

/* ---- Go-pattern CPU baseline ------------------------------------------ */

typedef struct { uint8_t *key; uint32_t klen; uint8_t *val; uint32_t vlen; } golike_pair;

typedef struct {
    int grammar;
    const uint8_t *base;
    const uint64_t *blk_off;
    const uint32_t *blk_len;
    uint64_t b0, b1;
    uint64_t recs;
} golike_job;

static void *golike_worker(void *arg) {
    golike_job *j = (golike_job *)arg;
    uint64_t recs = 0;
    for (uint64_t b = j->b0; b < j->b1; b++) {
        const uint8_t *p = j->base + j->blk_off[b];
        uint64_t n = j->blk_len[b], pos = 0;
        golike_pair *pairs = NULL;
        uint64_t np = 0, capp = 0;
        while (pos < n) {
            uint32_t kl = 0, vl;
            uint8_t *key = NULL;
            uint8_t lenbuf[4];
            if (j->grammar != ORA_GRAMMAR_V) {
                if (n - pos < 4) break;
                memcpy(lenbuf, p + pos, 4); /* binary.Read copies into a fresh buffer */
                kl = ld_u32le(lenbuf);
                if (kl > KEY_CAP || n - pos - 4 < kl) break;
                key = (uint8_t *)malloc(kl ? kl : 1);
                memcpy(key, p + pos + 4, kl);
                pos += 4 + (uint64_t)kl;
            }
            if (n - pos < 4) { free(key); break; }
            memcpy(lenbuf, p + pos, 4);
            vl = ld_u32le(lenbuf);
            if (n - pos - 4 < vl) { free(key); break; }
            uint8_t *val = (uint8_t *)malloc(vl ? vl : 1);
            memcpy(val, p + pos + 4, vl);
            pos += 4 + (uint64_t)vl;
            if (np == capp) { /* append growth */
                capp = capp ? capp * 2 : 1;
                pairs = (golike_pair *)realloc(pairs, capp * sizeof(golike_pair));
            }
            pairs[np].key = key; pairs[np].klen = kl;
            pairs[np].val = val; pairs[np].vlen = vl;
            np++;
        }
        recs += np;
        for (uint64_t i = 0; i < np; i++) { free(pairs[i].key); free(pairs[i].val); }
        free(pairs);
    }
    j->recs = recs;
    return NULL;
}

uint64_t ora_bench_decode_golike(int grammar, const uint8_t *base, const uint64_t *blk_off,
                                 const uint32_t *blk_len, uint64_t nblk, int threads) {
    if (threads < 1) threads = 1;
    golike_job *jobs = (golike_job *)calloc((size_t)threads, sizeof(golike_job));
    pthread_t *tids = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    for (int t = 0; t < threads; t++) {
        jobs[t].grammar = grammar; jobs[t].base = base;
        jobs[t].blk_off = blk_off; jobs[t].blk_len = blk_len;
        jobs[t].b0 = nblk * (uint64_t)t / (uint64_t)threads;
        jobs[t].b1 = nblk * (uint64_t)(t + 1) / (uint64_t)threads;
        if (threads == 1) golike_worker(&jobs[t]);
        else pthread_create(&tids[t], NULL, golike_worker, &jobs[t]);
    }
    uint64_t recs = 0;
    for (int t = 0; t < threads; t++) {
        if (threads > 1) pthread_join(tids[t], NULL);
        recs += jobs[t].recs;
    }
    free(jobs); free(tids);
    return recs;
}

/* ---- compaction merge: CompactAndMergeKVs (sstable/merge.go:42-94) ------ */

typedef struct {
    const uint8_t *bytes;
    const uint64_t *koff;
    const uint32_t *klen;
} merge_keys;

/* Go string comparison a < b: bytewise, a proper prefix sorts first. */
static int key_cmp(const merge_keys *m, uint32_t a, uint32_t b) {
    const uint32_t la = m->klen[a], lb = m->klen[b];
    const int c = memcmp(m->bytes + m->koff[a], m->bytes + m->koff[b], la < lb ? la : lb);
    if (c) return c;
    return la < lb ? -1 : la > lb ? 1 : 0;
}

/* stable merge sort of indices by key (ties keep input order) */
static void merge_sort_idx(const merge_keys *m, uint32_t *a, uint32_t *tmp, uint64_t n) {
    if (n < 2) return;
    const uint64_t h = n / 2;
    merge_sort_idx(m, a, tmp, h);
    merge_sort_idx(m, a + h, tmp, n - h);
    uint64_t i = 0, j = h, k = 0;
    while (i < h && j < n) tmp[k++] = key_cmp(m, a[j], a[i]) < 0 ? a[j++] : a[i++];
    while (i < h) tmp[k++] = a[i++];
    while (j < n) tmp[k++] = a[j++];
    memcpy(a, tmp, n * sizeof(uint32_t));
}

/* container/heap (Go standard library, heap.go): up / down with Less = key < */
static void goheap_up(const merge_keys *m, uint32_t *h, uint64_t j) {
    while (j > 0) {
        const uint64_t i = (j - 1) / 2;
        if (!(key_cmp(m, h[j], h[i]) < 0)) break;
        const uint32_t t = h[i]; h[i] = h[j]; h[j] = t;
        j = i;
    }
}

static void goheap_down(const merge_keys *m, uint32_t *h, uint64_t i, uint64_t n) {
    for (;;) {
        const uint64_t j1 = 2 * i + 1;
        if (j1 >= n) break;
        uint64_t j = j1;
        if (j1 + 1 < n && key_cmp(m, h[j1 + 1], h[j1]) < 0) j = j1 + 1;
        if (!(key_cmp(m, h[j], h[i]) < 0)) break;
        const uint32_t t = h[i]; h[i] = h[j]; h[j] = t;
        i = j;
    }
}

static const uint8_t kTombstone[13] = {0xEF, 0xBD, 0x9E, 'D', 'E', 'L', 'E', 'T',
                                       'E', 'D', 0xEF, 0xBD, 0x9E}; /* kv.go:29 "～DELETED～" */

uint64_t ora_merge_kvs(const uint8_t *bytes, const uint64_t *koff, const uint32_t *klen,
                       const uint64_t *voff, const uint32_t *vlen, uint64_t n, int level,
                       uint64_t threshold, int tie, uint32_t *out, uint64_t *starts,
                       uint64_t *nfiles) {
    merge_keys m = {bytes, koff, klen};
    uint32_t *order = (uint32_t *)malloc((n ? n : 1) * sizeof(uint32_t));
    uint32_t *tmp = (uint32_t *)malloc((n ? n : 1) * sizeof(uint32_t));
    if (tie == ORA_TIE_GOHEAP) {
        /* heap.Push each pair (merge.go:47-49), then heap.Pop until empty */
        for (uint64_t i = 0; i < n; i++) {
            tmp[i] = (uint32_t)i;
            goheap_up(&m, tmp, i);
        }
        for (uint64_t r = n; r > 0; r--) {
            const uint32_t t = tmp[0]; tmp[0] = tmp[r - 1]; tmp[r - 1] = t;
            goheap_down(&m, tmp, 0, r - 1);
            order[n - r] = tmp[r - 1];
        }
    } else {
        for (uint64_t i = 0; i < n; i++) order[i] = (uint32_t)i;
        merge_sort_idx(&m, order, tmp, n);
    }
    /* the loop of merge.go:57-91 over the pop order */
    uint64_t cnt = 0, nf = 0, size = 0;
    int64_t last = -1; /* lastWrittenKey: index of its pair, -1 = "" */
    starts[0] = 0;
    for (uint64_t t = 0; t < n; t++) {
        const uint32_t p = order[t];
        if (last >= 0 && klen[last] > 0 && key_cmp(&m, p, (uint32_t)last) == 0) continue;
        const int deleted = vlen[p] == 13 && memcmp(bytes + voff[p], kTombstone, 13) == 0;
        if (!deleted || level < 6) {
            out[cnt++] = p;
            size += 4 + (uint64_t)klen[p] + 4 + (uint64_t)vlen[p] + 8; /* kv.go:118-121 */
            last = p;
        }
        if (size >= threshold) { /* ShouldFlush, builder.go:40-42 */
            starts[++nf] = cnt;
            size = 0;
            last = -1;
        }
    }
    if (size > 0) starts[++nf] = cnt; /* merge.go:88-91 */
    *nfiles = nf;
    free(order);
    free(tmp);
    return cnt;
}

/* ---- batched SSTable.MayContain (CPU baseline) -------- */

static int go_strcmp(const uint8_t *a, uint64_t la, const uint8_t *b, uint64_t lb) {
    uint64_t n = la < lb ? la : lb;
    int c = n ? memcmp(a, b, n) : 0;
    if (c) return c;
    return la < lb ? -1 : la > lb ? 1 : 0;
}

/* SSTable.MayContain (sstable.go:300-305) of one decoded image: the key range
 * check, then Filter.Test (bloom.go:371-379) with the bits read from the
 * stored words.  A file whose header or filter did not decode answers 0. */
static uint8_t may_contain_one(const uint8_t *base, const ora_sst_meta *M, const uint8_t *key,
                               uint64_t kl) {
    if (M->stage == 1 || M->stage == 2) return 0;
    /* sstable.go:301: MinKey > key || MaxKey < key -> false */
    if (go_strcmp(base + M->min_key_off, M->min_key_len, key, kl) > 0 ||
        go_strcmp(base + M->max_key_off, M->max_key_len, key, kl) < 0)
        return 0;
    uint64_t h[4];
    ora_sum256(key, kl, h);
    uint8_t r = 1;
    for (uint64_t j = 0; j < M->filter_k && r; j++) {
        if (M->filter_m == 0) return 0; /* Go panics; the ABI answers 0 */
        const uint64_t q = ora_location(h, j) % M->filter_m;
        if (q >= M->filter_nbits) return 0;
        const uint8_t byte = base[M->filter_words_off + 8 * (q >> 6) + 7 - ((q & 63) >> 3)];
        r = (byte >> (q & 7)) & 1;
    }
    return r;
}

void ora_may_contain_batch(const uint8_t *img, const uint64_t *file_off, const ora_sst_meta *meta,
                           uint32_t nfile, const uint8_t *keys, const uint64_t *koff, uint64_t k0,
                           uint64_t k1, uint8_t *hit) {
    for (uint64_t i = k0; i < k1; i++) {
        const uint8_t *key = keys + koff[i];
        const uint64_t kl = koff[i + 1] - koff[i];
        for (uint32_t f = 0; f < nfile; f++)
            hit[(i - k0) * nfile + f] = may_contain_one(img + file_off[f], &meta[f], key, kl);
    }
}

void ora_level_may_contain(const uint8_t *img, const uint64_t *file_off, const ora_sst_meta *meta,
                           uint32_t nfile, const uint8_t *keys, const uint64_t *koff, uint64_t k0,
                           uint64_t k1, int32_t *table, uint8_t *may) {
    for (uint64_t i = k0; i < k1; i++) {
        const uint8_t *key = keys + koff[i];
        const uint64_t kl = koff[i + 1] - koff[i];
        /* sort.Search(len(sparseIndexes), f) (manager.go:186-188; Go sort.go:
         * i, j := 0, n; for i < j { h := int(uint(i+j) >> 1); if !f(h) { i = h + 1 }
         * else { j = h } }), f(h) = bytes.Compare(MinKey_h, key) > 0; a file whose
         * header did not decode has the zero Header, MinKey "" */
        uint32_t lo = 0, hi = nfile;
        while (lo < hi) {
            const uint32_t h = (uint32_t)(((uint64_t)lo + hi) >> 1);
            const ora_sst_meta *M = &meta[h];
            const int hdr = M->stage != 1;
            const int gt = hdr && go_strcmp(img + file_off[h] + M->min_key_off, M->min_key_len,
                                            key, kl) > 0;
            if (!gt) lo = h + 1;
            else hi = h;
        }
        uint32_t idx = lo;
        if (idx > 0) idx--; /* manager.go:189-191 */
        if (idx < nfile) {  /* manager.go:194-196: searchFromTable -> MayContain (:209-212) */
            table[i - k0] = (int32_t)idx;
            may[i - k0] = may_contain_one(img + file_off[idx], &meta[idx], key, kl);
        } else {            /* an empty level */
            table[i - k0] = -1;
            may[i - k0] = 0;
        }
    }
}

/* searchFromTable past MayContain (sstable/manager.go:209-223) on table t:
 * Iterator.Seek (sstable/block/index.go:157-181) over the table's decoded
 * IndexBlock, then Iterator.Value (sstable/iterator.go:34-46) ->
 * GetValueByOffset (sstable.go:271-296) -> Value.DecodeFrom (kv.go:181-200)
 * reading the file.  -> an ORA_GET_* code; the value's view on FOUND. */
static int32_t get_one(const uint8_t *img, const uint64_t *file_off, const uint64_t *file_len,
                       const ora_sst_meta *meta, const ora_desc *idx_desc, const int64_t *idx_val,
                       const uint64_t *idx_base, uint32_t t, const uint8_t *key, uint64_t kl,
                       uint64_t *val_off, uint32_t *val_len) {
    const uint8_t *file = img + file_off[t];
    const ora_desc *D = idx_desc + idx_base[t];
    const int64_t *V = idx_val + idx_base[t];
    const uint64_t n = meta[t].nidx;
    /* Seek: left, right := 0, len; for left < right { mid := left + (right-left)/2;
     * if Indexes[mid].Key < target { left = mid + 1 } else { right = mid } } */
    uint64_t left = 0, right = n;
    while (left < right) {
        const uint64_t mid = left + (right - left) / 2;
        if (go_strcmp(file + D[mid].rec_off + 4, D[mid].key_len, key, kl) < 0) left = mid + 1;
        else right = mid;
    }
    /* out of range or not an exact match: invalid, it.Valid() false -> (nil, nil) */
    if (left >= n || go_strcmp(file + D[left].rec_off + 4, D[left].key_len, key, kl) != 0)
        return ORA_GET_ABSENT;
    const int64_t off = V[left];
    if (off < 0) return ORA_GET_SEEK_FAILED; /* file.Seek: negative position */
    const uint64_t fl = file_len[t];
    const uint64_t rem = (uint64_t)off < fl ? fl - (uint64_t)off : 0;
    if (rem < 4) return ORA_GET_VALUE_LENGTH; /* binary.Read: EOF */
    const uint32_t vl = ld_u32le(file + off);
    if (vl > (1u << 30)) return ORA_GET_VALUE_TOO_LONG;
    if (rem - 4 < vl) return ORA_GET_VALUE_SHORT; /* io.ReadFull */
    *val_off = file_off[t] + (uint64_t)off;
    *val_len = vl;
    return ORA_GET_FOUND;
}

void ora_level_get(const uint8_t *img, const uint64_t *file_off, const uint64_t *file_len,
                   const ora_sst_meta *meta, const ora_desc *idx_desc, const int64_t *idx_val,
                   const uint64_t *idx_base, const uint8_t *keys, const uint64_t *koff, uint64_t k0,
                   uint64_t k1, const int32_t *table, const uint8_t *may, int32_t *res,
                   uint64_t *val_off, uint32_t *val_len) {
    for (uint64_t i = k0; i < k1; i++) {
        const uint64_t o = i - k0;
        res[o] = ORA_GET_ABSENT;
        val_off[o] = 0;
        val_len[o] = 0;
        if (!may[o] || table[o] < 0) continue; /* searchFromTable: !MayContain -> (nil, nil) */
        res[o] = get_one(img, file_off, file_len, meta, idx_desc, idx_val, idx_base, (uint32_t)table[o],
                         keys + koff[i], koff[i + 1] - koff[i], &val_off[o], &val_len[o]);
    }
}

/* Manager.searchFromLevel0 (sstable/manager.go:160-176): every level-0 table
 * in the Manager's order (newest first: addNewSSTables prepends,
 * manager.go:284-287), searchFromTable (:209-223) on each -- MayContain
 * (sstable.go:300-305), then Seek and the value -- and the first non-nil
 * value wins; an error ends the search (`return nil, err`).  table[o] = the
 * table that answered (FOUND or an error), -1 when none did. */
void ora_level0_get(const uint8_t *img, const uint64_t *file_off, const uint64_t *file_len,
                    const ora_sst_meta *meta, uint32_t nfile, const ora_desc *idx_desc,
                    const int64_t *idx_val, const uint64_t *idx_base, const uint8_t *keys,
                    const uint64_t *koff, uint64_t k0, uint64_t k1, int32_t *table, int32_t *res,
                    uint64_t *val_off, uint32_t *val_len) {
    for (uint64_t i = k0; i < k1; i++) {
        const uint64_t o = i - k0;
        const uint8_t *key = keys + koff[i];
        const uint64_t kl = koff[i + 1] - koff[i];
        res[o] = ORA_GET_ABSENT;
        table[o] = -1;
        val_off[o] = 0;
        val_len[o] = 0;
        for (uint32_t t = 0; t < nfile; t++) {
            if (!may_contain_one(img + file_off[t], &meta[t], key, kl)) continue; /* (nil, nil) */
            const int32_t r = get_one(img, file_off, file_len, meta, idx_desc, idx_val, idx_base, t, key,
                                      kl, &val_off[o], &val_len[o]);
            if (r == ORA_GET_ABSENT) continue; /* val == nil: the next table */
            res[o] = r;
            table[o] = (int32_t)t;
            break;
        }
    }
}

/* ---- config 1 from a file, the reference's syscall pattern --------------- */
/* SSTable.DecodeFrom(path) (sstable.go:87-127) then GetDataBlockFromFile(path)
 * (sstable.go:227-268) over an unbuffered *os.File: every binary.Read and
 * io.ReadFull is one read(2) of exactly the field (Header keys header.go:40-52
 * via Key.DecodeFrom kv.go:124-139; the filter length and block bloom.go:
 * 453-469; the footer's two 16-byte handles footer.go:58-86 after a Stat and
 * a Seek; per index entry 4 + key + 8 bytes index.go:70-98; per value 4 +
 * value bytes data.go:58-76 under io.LimitReader), a fresh heap buffer per key
 * and value, append-grown entry slices and the positional join into an
 * append-grown pair slice.  Test infrastructure: the file-backed CPU
 * baseline of config 1.  -> pairs, or < 0. */
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

static int rd_full(int fd, void *p, uint64_t n) {  /* io.ReadFull: one read(2) */
    uint8_t *q = (uint8_t *)p;
    while (n) {
        const ssize_t r = read(fd, q, n);
        if (r <= 0) return -1;
        q += r;
        n -= (uint64_t)r;
    }
    return 0;
}

typedef struct { uint8_t *p; uint32_t n; } ora_buf;
typedef struct { ora_buf *a; uint64_t len, cap; } ora_bufvec;

static void bv_push(ora_bufvec *v, ora_buf b) {     /* Go append growth */
    if (v->len == v->cap) {
        v->cap = v->cap ? (v->cap < 256 ? 2 * v->cap : v->cap + v->cap / 4) : 1;
        v->a = (ora_buf *)realloc(v->a, v->cap * sizeof(ora_buf));
    }
    v->a[v->len++] = b;
}

static void bv_free(ora_bufvec *v) {
    for (uint64_t i = 0; i < v->len; i++) free(v->a[i].p);
    free(v->a);
}

static int rd_key(int fd, ora_buf *k) {             /* Key.DecodeFrom kv.go:124-139 */
    uint32_t kl;
    if (rd_full(fd, &kl, 4)) return -1;
    k->p = (uint8_t *)malloc(kl ? kl : 1);
    k->n = kl;
    if (rd_full(fd, k->p, kl)) {  /* the caller never owns a key it did not get */
        free(k->p);
        k->p = NULL;
        return -1;
    }
    return 0;
}

int64_t ora_sst_decode_file(const char *path) {
    /* SSTable.DecodeFrom: header, filter, footer, index */
    int fd = open(path, O_RDONLY);
    if (fd < 0) return -1;
    ora_buf mn = {0}, mx = {0};
    int64_t rc = -2;
    ora_bufvec ikeys = {0};
    uint64_t *ioffs = NULL, nio = 0, cio = 0;
    int64_t fo[4];
    if (rd_key(fd, &mn) || rd_key(fd, &mx)) goto out;
    uint64_t L;
    if (rd_full(fd, &L, 8)) goto out;
    uint8_t *fb = (uint8_t *)malloc(L ? L : 1);
    if (rd_full(fd, fb, L) || L < 24) { free(fb); goto out; }
    {   /* UnmarshalBinary: m, k, then the bitset words into a fresh slice */
        const uint64_t nb = ld_u64be(fb + 16), nw = nb / 64 + ((nb & 63) != 0);
        if (nw > (L - 24) / 8) { free(fb); goto out; }
        uint64_t *words = (uint64_t *)malloc((nw ? nw : 1) * 8);
        for (uint64_t i = 0; i < nw; i++) words[i] = ld_u64be(fb + 24 + 8 * i);
        free(words);
        free(fb);
    }
    struct stat st;
    if (fstat(fd, &st) || st.st_size < 32 || lseek(fd, st.st_size - 32, SEEK_SET) < 0) goto out;
    if (rd_full(fd, fo, 16) || rd_full(fd, fo + 2, 16)) goto out;  /* two Handles */
    if (fo[2] < 0 || fo[3] < 0 || lseek(fd, fo[2], SEEK_SET) < 0) goto out;
    for (int64_t tot = 0; tot < fo[3];) {               /* IndexBlock.DecodeFrom */
        ora_buf k;
        if (rd_key(fd, &k)) goto out;
        bv_push(&ikeys, k);
        int64_t o;
        if (rd_full(fd, &o, 8)) goto out;
        if (nio == cio) {
            cio = cio ? (cio < 256 ? 2 * cio : cio + cio / 4) : 1;
            ioffs = (uint64_t *)realloc(ioffs, cio * 8);
        }
        ioffs[nio++] = (uint64_t)o;
        tot += 4 + (int64_t)k.n + 8;
        if (tot > fo[3]) goto out;
    }
    close(fd);
    /* GetDataBlockFromFile: open, DecodeDataBlock, GetKeyValuePairs */
    fd = open(path, O_RDONLY);
    if (fd < 0) { fd = -1; goto out; }
    ora_bufvec vals = {0};
    if (fo[0] < 0 || lseek(fd, fo[0], SEEK_SET) < 0) goto out;
    {
        uint64_t left = fo[1] > 0 ? (uint64_t)fo[1] : ~0ull;  /* io.LimitReader */
        for (;;) {                                      /* DataBlock.DecodeFrom */
            uint32_t vl;
            uint64_t got = 0;
            while (got < 4 && left) {                   /* binary.Read: ReadFull of 4 */
                const uint64_t want = 4 - got < left ? 4 - got : left;
                const ssize_t r = read(fd, (uint8_t *)&vl + got, want);
                if (r <= 0) break;
                got += (uint64_t)r;
                left -= (uint64_t)r;
            }
            if (got == 0) break;                        /* io.EOF: a clean stop */
            if (got < 4 || left < vl) { bv_free(&vals); goto out; }
            ora_buf v = {(uint8_t *)malloc(vl ? vl : 1), vl};
            if (rd_full(fd, v.p, vl)) { free(v.p); bv_free(&vals); goto out; }
            left -= vl;
            bv_push(&vals, v);
        }
    }
    if (vals.len == 0 || ikeys.len == 0) rc = 0;
    else if (vals.len != ikeys.len) rc = -3;            /* mismatched entries */
    else {
        typedef struct { ora_buf k, v; } pair;          /* pairs := make(.., 0); append */
        pair *pairs = NULL;
        uint64_t np = 0, cp = 0;
        for (uint64_t i = 0; i < vals.len; i++) {
            if (np == cp) {
                cp = cp ? (cp < 256 ? 2 * cp : cp + cp / 4) : 1;
                pairs = (pair *)realloc(pairs, cp * sizeof(pair));
            }
            pairs[np].k = ikeys.a[i];
            pairs[np++].v = vals.a[i];
        }
        free(pairs);
        rc = (int64_t)np;
    }
    bv_free(&vals);
out:
    if (fd >= 0) close(fd);
    free(mn.p);
    free(mx.p);
    bv_free(&ikeys);
    free(ioffs);
    return rc;
}
