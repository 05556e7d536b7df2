/* sanitize_main.c -- host fuzz driver for the oracle under ASan + UBSan.
 *
 * Test infrastructure only (built by `make -C oracle sanitize`, run by
 * tests/test_oracle_sanitize.py): every input buffer is malloc'd at its
 * exact size, so a read one byte past a block, key, filter or image is an
 * ASan report.  Covers the record decoders (valid, truncated, random and
 * giant-length blocks of all three grammars), materialization, encode ->
 * decode round trips, sum256 over lengths 0..300, bloom add/test, filter
 * block encode/decode (incl. truncations), .sst build -> decode (incl.
 * truncated and bit-flipped images), the batched MayContain and the merge in
 * both tie modes.  Exits 0 when every self-check holds. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "lsm_oracle.h"

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void) {
    rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17;
    return rs;
}
static uint32_t rn(uint32_t n) { return n ? (uint32_t)(rnd() % n) : 0; }

#define CHECK(c) do { if (!(c)) { fprintf(stderr, "check failed %s:%d: %s\n", __FILE__, __LINE__, #c); exit(1); } } while (0)

static void put32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }
static void put64(uint8_t *p, uint64_t v) { memcpy(p, &v, 8); }

/* one random block of grammar g with nrec records; returns its size */
static size_t make_block(int g, uint8_t *b, uint32_t nrec, uint32_t kmax, uint32_t vmax) {
    size_t n = 0;
    for (uint32_t r = 0; r < nrec; r++) {
        const uint32_t kl = rn(kmax + 1), vl = rn(vmax + 1);
        if (g != 0) { put32(b + n, kl); n += 4; for (uint32_t i = 0; i < kl; i++) b[n++] = (uint8_t)rnd(); }
        if (g == 2) { put64(b + n, rnd()); n += 8; continue; }
        put32(b + n, vl); n += 4;
        for (uint32_t i = 0; i < vl; i++) b[n++] = (uint8_t)rnd();
    }
    return n;
}

static void fuzz_decode(void) {
    uint8_t *tmp = malloc(1 << 20);
    for (int it = 0; it < 30000; it++) {
        const int g = it % 3;
        size_t n = make_block(g, tmp, rn(40), 40, 300);
        switch (rn(5)) {
        case 0: n = n ? rn((uint32_t)n) : 0; break;                          /* truncated */
        case 1: for (int i = 0; i < 4 && n; i++) tmp[rn((uint32_t)n)] = (uint8_t)rnd(); break;
        case 2: if (n >= 4) put32(tmp + 4 * rn((uint32_t)(n / 4)), 0xFFFFFFF0u); break;
        case 3: n += rn(4); break;                                           /* 1-3 trailing bytes */
        default: break;
        }
        uint8_t *blk = malloc(n ? n : 1);
        memcpy(blk, tmp, n);
        ora_desc *d = malloc(sizeof(ora_desc) * (n / 4 + 1));
        int64_t *iv = malloc(8 * (n / 4 + 1));
        uint32_t nrec = 0;
        ora_decode_block(g, blk, 0, n, d, iv, n / 4 + 1, &nrec);
        uint64_t kb = 0, vb = 0;
        for (uint32_t i = 0; i < nrec; i++) {
            CHECK(d[i].rec_off < n);
            kb += d[i].key_len;
            vb += d[i].val_len;
        }
        uint8_t *ka = malloc(kb + 1), *va = malloc(vb + 1);
        uint64_t vbytes = 0;
        const uint64_t kbytes = ora_materialize(g, blk, d, nrec, ka, va, &vbytes);
        CHECK(g == 0 ? kbytes == 0 : kbytes == kb);
        free(ka); free(va); free(blk); free(d); free(iv);
    }
    free(tmp);
}

static void fuzz_encode(void) {
    for (int it = 0; it < 3000; it++) {
        const int g = it % 3;
        const uint32_t n = rn(50);
        uint64_t *koff = malloc(8 * (n + 1)), *voff = malloc(8 * (n + 1));
        koff[0] = voff[0] = 0;
        for (uint32_t i = 0; i < n; i++) {
            koff[i + 1] = koff[i] + rn(30);
            voff[i + 1] = voff[i] + rn(200);
        }
        uint8_t *keys = malloc(koff[n] + 1), *vals = malloc(voff[n] + 1);
        for (uint64_t i = 0; i < koff[n]; i++) keys[i] = (uint8_t)rnd();
        for (uint64_t i = 0; i < voff[n]; i++) vals[i] = (uint8_t)rnd();
        int64_t *xo = malloc(8 * (n + 1));
        for (uint32_t i = 0; i < n; i++) xo[i] = (int64_t)rnd();
        const uint64_t sz = ora_encoded_size(g, koff, voff, 0, n);
        uint8_t *out = malloc(sz ? sz : 1);
        CHECK(ora_encode_records(g, keys, koff, vals, voff, 0, n, xo, out) == sz);
        ora_desc *d = malloc(sizeof(ora_desc) * (n + 1));
        uint32_t nrec = 0;
        CHECK(ora_decode_block(g, out, 0, sz, d, NULL, n + 1, &nrec) == ORA_OK && nrec == n);
        free(keys); free(vals); free(koff); free(voff); free(xo); free(out); free(d);
    }
}

static void fuzz_bloom_sst(void) {
    CHECK(ora_mmh3_verification() == 0x6384BA69u);
    for (uint32_t len = 0; len <= 300; len++) {
        uint8_t *k = malloc(len ? len : 1);
        for (uint32_t i = 0; i < len; i++) k[i] = (uint8_t)(i * 7 + len);
        uint64_t h[4];
        ora_sum256(k, len, h);
        free(k);
    }
    const uint64_t ms[] = {1, 63, 64, 65, 1000, 100003};
    for (int mi = 0; mi < 6; mi++) {
        const uint64_t m = ms[mi], k = 1 + rn(20), nw = (m + 63) / 64;
        uint64_t *w = calloc(nw, 8);
        uint8_t key[24];
        for (int i = 0; i < 200; i++) {
            for (int j = 0; j < 24; j++) key[j] = (uint8_t)rnd();
            const uint32_t kl = rn(25);
            ora_bloom_add(w, m, k, key, kl);
            CHECK(ora_bloom_test(w, m, k, key, kl));
        }
        const uint64_t fb = ora_filter_block_size(m);
        uint8_t *blk = malloc(fb);
        CHECK(ora_filter_encode(w, m, k, blk) == fb);
        for (int cut = 0; cut < 8; cut++) {
            const uint64_t n = cut ? rn((uint32_t)fb) : fb;
            uint8_t *in = malloc(n ? n : 1);
            memcpy(in, blk, n);
            uint64_t m2, k2, nb, used;
            uint64_t *w2 = calloc(nw + 1, 8);
            const int rc = ora_filter_decode(in, n, &m2, &k2, &nb, w2, nw + 1, &used);
            if (!cut) CHECK(rc == 0 && m2 == m && k2 == k && used == fb);
            free(in); free(w2);
        }
        free(w); free(blk);
    }
    /* .sst build -> decode, then truncated / bit-flipped images */
    for (int it = 0; it < 40; it++) {
        const uint32_t n = rn(300);
        uint64_t *koff = malloc(8 * (n + 1)), *voff = malloc(8 * (n + 1));
        koff[0] = voff[0] = 0;
        for (uint32_t i = 0; i < n; i++) { koff[i + 1] = koff[i] + 16; voff[i + 1] = voff[i] + rn(120); }
        uint8_t *keys = malloc(koff[n] + 1), *vals = malloc(voff[n] + 1);
        for (uint32_t i = 0; i < n; i++) snprintf((char *)keys + 16 * i, 17, "k%015u", i);
        for (uint64_t i = 0; i < voff[n]; i++) vals[i] = (uint8_t)rnd();
        const uint64_t m = 1000 + rn(5000), k = 1 + rn(16);
        const uint64_t sz = ora_sst_image_size(koff, voff, 0, n, m);
        uint8_t *img = malloc(sz);
        int64_t foot[4];
        CHECK(ora_build_sst(keys, koff, vals, voff, 0, n, m, k, img, foot) == sz);
        for (int v = 0; v < 6; v++) {
            uint64_t len = sz;
            uint8_t *im = malloc(sz);
            memcpy(im, img, sz);
            if (v == 1) len = rn((uint32_t)sz);
            if (v >= 2) im[rn((uint32_t)sz)] ^= (uint8_t)(1u << rn(8));
            uint8_t *cp = malloc(len ? len : 1);
            memcpy(cp, im, len);
            ora_sst_meta meta;
            ora_desc *id = malloc(sizeof(ora_desc) * (len / 4 + 1)), *dd = malloc(sizeof(ora_desc) * (len / 4 + 1));
            int64_t *iv = malloc(8 * (len / 4 + 1));
            const int rc = ora_sst_decode(cp, len, &meta, id, iv, len / 4 + 1, dd, len / 4 + 1);
            if (v == 0) CHECK(rc == 0 && meta.ndata == n && meta.nidx == n);
            if (v == 0 && n) {
                uint64_t fo = 0;
                uint8_t *hit = malloc(2 * (size_t)n);
                ora_may_contain_batch(cp, &fo, &meta, 1, keys, koff, 0, n, hit);
                for (uint32_t i = 0; i < n; i++) CHECK(hit[i] == 1);
                free(hit);
            }
            free(cp); free(im); free(id); free(dd); free(iv);
        }
        free(img); free(keys); free(vals); free(koff); free(voff);
    }
}

static void fuzz_merge(void) {
    for (int it = 0; it < 200; it++) {
        const uint32_t n = rn(400);
        uint64_t *koff = malloc(8 * (n + 1)), *voff = malloc(8 * (n + 1));
        uint32_t *klen = malloc(4 * (n + 1)), *vlen = malloc(4 * (n + 1));
        uint8_t *bytes = malloc(32 * (size_t)n + 1);
        uint64_t p = 0;
        for (uint32_t i = 0; i < n; i++) {
            klen[i] = 1 + rn(6);
            koff[i] = p;
            for (uint32_t j = 0; j < klen[i]; j++) bytes[p++] = (uint8_t)('a' + rn(3));
            vlen[i] = rn(9);
            voff[i] = p;
            for (uint32_t j = 0; j < vlen[i]; j++) bytes[p++] = (uint8_t)rnd();
        }
        uint32_t *out = malloc(4 * (n + 1));
        uint64_t *starts = malloc(8 * (n + 2)), nf = 0;
        for (int tie = 0; tie < 2; tie++)
            CHECK(ora_merge_kvs(bytes, koff, klen, voff, vlen, n, rn(7), rn(400), tie, out, starts, &nf) <= n);
        free(koff); free(voff); free(klen); free(vlen); free(bytes); free(out); free(starts);
    }
}

int main(void) {
    fuzz_decode();
    fuzz_encode();
    fuzz_bloom_sst();
    fuzz_merge();
    printf("oracle sanitizer run ok\n");
    return 0;
}
