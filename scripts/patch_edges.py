# A/B variant: the region streams' chunk-edge segments (the first and last 16 bytes of a
# stream, partly outside it) read their four dwords from LDS unconditionally, funnel them as
# the whole segments do, and store only the bytes inside the stream -- instead of one
# conditional LDS byte read per byte (sixteen waits in a row on every edge iteration).
s = open('encode.hip').read()
old = '''        } else {
            gptr_t<uint8_t> db = (gptr_t<uint8_t>)(dA + e);
            for (uint32_t b = 0; b < 16; b++) {
                const int32_t u = u0 + (int32_t)b;
                if (u >= 0 && (uint32_t)u < tot) db[b] = ob[u];
            }
        }'''
assert old in s
s = s.replace(old, '''        } else {
            // edge segment: the same funnels (LDS reads never fault; bytes
            // outside the stream are read and dropped), stores inside only
            gptr_t<uint8_t> db = (gptr_t<uint8_t>)(dA + e);
            const uint32_t q = q0 + 4 * e;
            uint32_t wd[4];
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) wd[k] = funnel(lds[q + k], lds[q + k + 1], sh);
#pragma unroll
            for (uint32_t b = 0; b < 16; b++) {
                const int32_t u = u0 + (int32_t)b;
                if (u >= 0 && (uint32_t)u < tot) db[b] = (uint8_t)(wd[b >> 2] >> (8 * (b & 3)));
            }
        }''')
old = '''        } else {
            gptr_t<uint8_t> db = (gptr_t<uint8_t>)(dA + e);
            for (uint32_t k = 0; k < 4; k++) {
                const int32_t u = u0 + 4 * (int32_t)k;
                if (u >= 0 && u + 4 <= tot) {
                    const uint32_t q = q0 + 4 * e + k;
                    *(gptr_t<uint32_t>)(db + 4 * k) = funnel(img[q], img[q + 1], R.sh);
                } else {
                    for (uint32_t b = 0; b < 4; b++)
                        if (u + (int32_t)b >= 0 && u + (int32_t)b < tot) db[4 * k + b] = ob[u + b];
                }
            }
        }'''
assert old in s
s = s.replace(old, '''        } else {
            // edge segment: all four funnels first (LDS reads never fault;
            // bytes outside the stream are read and dropped), then the stores
            gptr_t<uint8_t> db = (gptr_t<uint8_t>)(dA + e);
            uint32_t wd[4];
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) {
                const uint32_t q = q0 + 4 * e + k;
                wd[k] = funnel(img[q], img[q + 1], R.sh);
            }
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) {
                const int32_t u = u0 + 4 * (int32_t)k;
                if (u >= 0 && u + 4 <= tot) {
                    *(gptr_t<uint32_t>)(db + 4 * k) = wd[k];
                } else {
#pragma unroll
                    for (uint32_t b = 0; b < 4; b++)
                        if (u + (int32_t)b >= 0 && u + (int32_t)b < tot)
                            db[4 * k + b] = (uint8_t)(wd[k] >> (8 * b));
                }
            }
        }''')
open('encode.hip', 'w').write(s)
print('ok edges')
