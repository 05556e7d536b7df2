# A/B variant (on the slot-grouped all-tables path): the hit matrix's rows written once by
# classify after its searches, with each candidate's 1 in place (the candidates in LDS,
# aliasing the scan's scratch row), and the test writing only the 0s of failed candidates.
s = open('encode.hip').read()
old = '''    {   // the workgroup's rows of the hit matrix start at 0 (16-byte stores
        // while the key loads are in flight)
        const uint64_t r0 = k_begin + (uint64_t)blockIdx.x * kMcGroupProbes;
        const uint64_t r1 = r0 + kMcGroupProbes < nkeys ? r0 + kMcGroupProbes : nkeys;
        uint8_t *z = hit + r0 * nfile;
        const uint64_t nz = (r1 - r0) * nfile;
        const uint64_t head = ((16 - ((uintptr_t)z & 15)) & 15) < nz ? ((16 - ((uintptr_t)z & 15)) & 15) : nz;
        const uint64_t n16 = (nz - head) / 16, tail = head + 16 * n16;
        if (threadIdx.x < head) z[threadIdx.x] = 0;
        uint4 *z16 = reinterpret_cast<uint4 *>(z + head);
        for (uint64_t x = threadIdx.x; x < n16; x += kMcGroupThreads) z16[x] = make_uint4(0, 0, 0, 0);
        if (tail + threadIdx.x < nz) z[tail + threadIdx.x] = 0;
    }
'''
assert old in s
s = s.replace(old, '')
old = '''            if (r >= 0) {  // only candidates are ever tested
                cand[p] = lo - 1;
                rank[p] = atomicAdd(&lh[lo - 1], 1u);
                sum256_pre(kp, kl[p], f0[p], f1[p], hh[p]);
            }
        }
    }
    __syncthreads();'''
assert old in s
s = s.replace(old, '''            if (r >= 0) {  // only candidates are ever tested
                cand[p] = lo - 1;
                rank[p] = atomicAdd(&lh[lo - 1], 1u);
                sum256_pre(kp, kl[p], f0[p], f1[p], hh[p]);
            }
        }
    }
    {   // the workgroup's rows of the hit matrix, written once: 0 except the
        // candidate's 1 (the test clears it when a bit is 0), 16-byte stores;
        // the candidates through LDS (the scan's row, free until the scan)
        uint16_t *scand = reinterpret_cast<uint16_t *>(part);
#pragma unroll
        for (uint32_t p = 0; p < kMcGroupPer; p++)
            scand[p * kMcGroupThreads + t] = cand[p] == kMcNone ? (uint16_t)0xFFFFu : (uint16_t)cand[p];
        __syncthreads();
        const uint64_t r0 = k_begin + (uint64_t)blockIdx.x * kMcGroupProbes;
        const uint64_t r1 = r0 + kMcGroupProbes < nkeys ? r0 + kMcGroupProbes : nkeys;
        uint8_t *z = hit + r0 * nfile;
        const uint32_t nz = (uint32_t)((r1 - r0) * nfile);  // <= 2,048 rows x 2,048 files
        const uint32_t mis = (uint32_t)((uintptr_t)z & 15);
        const uint32_t head = ((16 - mis) & 15) < nz ? ((16 - mis) & 15) : nz;
        const uint32_t n16 = (nz - head) / 16, tail = head + 16 * n16;
        auto one_at = [&](uint32_t o) -> uint32_t {  // byte o of the rows: the candidate's 1
            const uint32_t row = o / nfile;
            const uint32_t c = scand[row];
            return c != 0xFFFFu && row * nfile + c == o ? 1u : 0u;
        };
        if (t < head) z[t] = (uint8_t)one_at(t);
        u32x4 *z16 = reinterpret_cast<u32x4 *>(z + head);
        for (uint32_t x = t; x < n16; x += kMcGroupThreads) {
            const uint32_t o = head + 16 * x;
            uint32_t wd[4] = {0, 0, 0, 0};
            for (uint32_t row = o / nfile; row * nfile < o + 16; row++) {
                const uint32_t c = scand[row];
                const uint32_t at = row * nfile + c;
                if (c != 0xFFFFu && at >= o && at < o + 16) wd[(at - o) >> 2] |= 1u << (8 * ((at - o) & 3));
            }
            z16[x] = u32x4{wd[0], wd[1], wd[2], wd[3]};
        }
        if (tail + t < nz) z[tail + t] = (uint8_t)one_at(tail + t);
    }
    __syncthreads();''')
old = '''        if (Matrix) may[(k_begin + id) * nfile + f] = (uint8_t)r;'''
assert old in s
s = s.replace(old, '''        if (Matrix) {
            if (!r) may[(k_begin + id) * nfile + f] = 0;  // classify wrote the 1
        }''')
open('encode.hip', 'w').write(s)
print('ok fill2')
