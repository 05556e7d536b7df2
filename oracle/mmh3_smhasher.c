/*
 * mmh3_smhasher.c — independent MurmurHash3_x64_128 (Austin Appleby's
 * SMHasher reference algorithm, public domain), used ONLY to pin the
 * go-lsm sum256 restatement the way sstable/bloom/murmur_test.go:12-70
 * pins digest128.sum256 against github.com/twmb/murmur3 v1.1.8
 * (sum256(d) == (MMH3_128(d), MMH3_128(d || 0x01))).
 * This implementation is itself pinned by SMHasher's published
 * verification value for MurmurHash3_x64_128: 0x6384BA69.
 * TEST INFRASTRUCTURE ONLY.
 */
#include <stdint.h>
#include <string.h>

#include "lsm_oracle.h"

static uint64_t getblock(const uint8_t *p, uint64_t i) {
    uint64_t v;
    memcpy(&v, p + 8 * i, 8); /* x86-64 host: little-endian */
    return v;
}

static uint64_t rot(uint64_t x, int8_t r) { return (x << r) | (x >> (64 - r)); }

static uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}

void ora_mmh3_x64_128(const void *key, uint64_t len, uint32_t seed, uint64_t out[2]) {
    const uint8_t *data = (const uint8_t *)key;
    const uint64_t nblocks = len / 16;
    uint64_t h1 = seed, h2 = seed;
    const uint64_t c1 = 0x87c37b91114253d5ULL;
    const uint64_t c2 = 0x4cf5ad432745937fULL;

    for (uint64_t i = 0; i < nblocks; i++) {
        uint64_t k1 = getblock(data, i * 2 + 0);
        uint64_t k2 = getblock(data, i * 2 + 1);
        k1 *= c1; k1 = rot(k1, 31); k1 *= c2; h1 ^= k1;
        h1 = rot(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
        k2 *= c2; k2 = rot(k2, 33); k2 *= c1; h2 ^= k2;
        h2 = rot(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
    }

    const uint8_t *tail = data + nblocks * 16;
    uint64_t k1 = 0, k2 = 0;
    switch (len & 15) {
    case 15: k2 ^= ((uint64_t)tail[14]) << 48; /* fallthrough */
    case 14: k2 ^= ((uint64_t)tail[13]) << 40; /* fallthrough */
    case 13: k2 ^= ((uint64_t)tail[12]) << 32; /* fallthrough */
    case 12: k2 ^= ((uint64_t)tail[11]) << 24; /* fallthrough */
    case 11: k2 ^= ((uint64_t)tail[10]) << 16; /* fallthrough */
    case 10: k2 ^= ((uint64_t)tail[9]) << 8;   /* fallthrough */
    case 9:
        k2 ^= ((uint64_t)tail[8]) << 0;
        k2 *= c2; k2 = rot(k2, 33); k2 *= c1; h2 ^= k2;
        /* fallthrough */
    case 8: k1 ^= ((uint64_t)tail[7]) << 56; /* fallthrough */
    case 7: k1 ^= ((uint64_t)tail[6]) << 48; /* fallthrough */
    case 6: k1 ^= ((uint64_t)tail[5]) << 40; /* fallthrough */
    case 5: k1 ^= ((uint64_t)tail[4]) << 32; /* fallthrough */
    case 4: k1 ^= ((uint64_t)tail[3]) << 24; /* fallthrough */
    case 3: k1 ^= ((uint64_t)tail[2]) << 16; /* fallthrough */
    case 2: k1 ^= ((uint64_t)tail[1]) << 8;  /* fallthrough */
    case 1:
        k1 ^= ((uint64_t)tail[0]) << 0;
        k1 *= c1; k1 = rot(k1, 31); k1 *= c2; h1 ^= k1;
    }

    h1 ^= len; h2 ^= len;
    h1 += h2; h2 += h1;
    h1 = fmix64(h1); h2 = fmix64(h2);
    h1 += h2; h2 += h1;
    out[0] = h1;
    out[1] = h2;
}

/* SMHasher VerificationTest (KeysetTest.cpp): hash keys {}, {0}, {0,1}, ...
 * of lengths 0..255 with seed 256-i, hash the concatenated digests with seed
 * 0, and read the first 4 bytes little-endian. */
uint32_t ora_mmh3_verification(void) {
    uint8_t key[256];
    uint8_t hashes[16 * 256];
    uint64_t fin[2];
    for (int i = 0; i < 256; i++) {
        uint64_t o[2];
        key[i] = (uint8_t)i;
        ora_mmh3_x64_128(key, (uint64_t)i, (uint32_t)(256 - i), o);
        memcpy(hashes + 16 * i, o, 16);
    }
    ora_mmh3_x64_128(hashes, sizeof(hashes), 0, fin);
    uint8_t b[16];
    memcpy(b, fin, 16);
    return (uint32_t)b[0] | (uint32_t)b[1] << 8 | (uint32_t)b[2] << 16 | (uint32_t)b[3] << 24;
}
