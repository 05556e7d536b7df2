# A/B variant (on the source after the bit-read change): the level test loop with two
# probes per thread per iteration.
s = open('encode.hip').read()
b = s.index('''    uint32_t q = t, id = 0;
    u32x4 x = {0, 0, 0, 0}, y = {0, 0, 0, 0};
    if (q < total) {  // the first probe's hash in flight during the fill''')
e = s.index('''// More tables than the LDS search holds''')
new = r'''    constexpr uint32_t U = 2;  // probes per thread per iteration
    uint32_t q = t, id[U] = {};
    u32x4 x[U] = {}, y[U] = {};
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {  // the first probes' hashes in flight during the fill
        const uint32_t qu = q + u * kLvThreads;
        if (qu < total) {
            const uint64_t sl = slot_of(qu);
            id[u] = w.ids[sl];
            x[u] = w.rec[sl];
            if (!compact) y[u] = w.ext[sl];
        }
    }
    const uint8_t *src = img + F.words_at;
    uint32_t delta;
    const uint64_t in_lds = stage_filter(src, F.nbits, fbytes, kMcLdsBytes, f, delta);
    __asm__ __volatile__("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint8_t *lb = fbytes + delta;
    while (q < total) {
        const uint32_t qn = q + U * kLvThreads;
        uint32_t idn[U] = {};
        u32x4 xn[U] = {}, yn[U] = {};
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint32_t qu = qn + u * kLvThreads;
            if (qu < total) {
                const uint64_t sl = slot_of(qu);
                idn[u] = w.ids[sl];
                xn[u] = w.rec[sl];
                if (!compact) yn[u] = w.ext[sl];
            }
        }
        uint32_t r[U];
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            if (compact) {
                r[u] = filter_test_rec(F, unpack_hash_rec(x[u], m32, c64), m32, lb, in_lds, src);
            } else {
                const uint64_t h[4] = {(uint64_t)x[u].y << 32 | x[u].x, (uint64_t)x[u].w << 32 | x[u].z,
                                       (uint64_t)y[u].y << 32 | y[u].x, (uint64_t)y[u].w << 32 | y[u].z};
                r[u] = filter_test(F, h, lb, in_lds, src);
            }
        }
#pragma unroll
        for (uint32_t u = 0; u < U; u++)
            if (q + u * kLvThreads < total) may[k_begin + id[u]] = (uint8_t)r[u];
        q = qn;
#pragma unroll
        for (uint32_t u = 0; u < U; u++) { id[u] = idn[u]; x[u] = xn[u]; y[u] = yn[u]; }
    }
}

'''
s = s[:b] + new + s[e:]
open('encode.hip', 'w').write(s)
print('ok ilp2')
