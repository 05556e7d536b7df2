# A/B variant: the all-tables hit matrix's rows written once, with the candidate's 1 in
# place (mc_classify_kernel fills the workgroup's rows after its searches, from the
# candidates in LDS), so mc_scatter_kernel no longer stores a byte per candidate.
s = open('encode.hip').read()
old = '''    {   // the workgroup's rows of the hit matrix start at 0 (16-byte stores
        // while the key loads are in flight)
        const uint64_t r0 = (uint64_t)blockIdx.x * kMcGroupProbes;
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
old = '''    __shared__ uint4 slo[kMcMaxFiles], shi[kMcMaxFiles];
    __shared__ uint32_t lh[kMcMaxFiles];
    if (!w.flag[0]) return;'''
assert old in s
s = s.replace(old, '''    __shared__ uint4 slo[kMcMaxFiles], shi[kMcMaxFiles];
    __shared__ uint32_t lh[kMcMaxFiles];
    __shared__ uint16_t scand[kMcGroupProbes];  // candidate of each probe (0xFFFF: none)
    if (!w.flag[0]) return;''')
old = '''        if (i >= nkeys) break;
        const uint8_t *kp = keys + k0[p];'''
assert old in s
s = s.replace(old, '''        if (i >= nkeys) break;
        scand[p * kMcGroupThreads + threadIdx.x] = 0xFFFFu;
        const uint8_t *kp = keys + k0[p];''')
old = '''        w.cand[i] = c;
    }
    __syncthreads();'''
assert old in s
s = s.replace(old, '''        w.cand[i] = c;
        if (c != kMcNone) scand[p * kMcGroupThreads + threadIdx.x] = (uint16_t)c;
    }
    __syncthreads();
    {   // the workgroup's rows of the hit matrix, written once: 0 except the
        // candidate's 1 (the test clears it when a bit is 0), 16-byte stores
        const uint64_t r0 = (uint64_t)blockIdx.x * kMcGroupProbes;
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
        if (threadIdx.x < head) z[threadIdx.x] = (uint8_t)one_at(threadIdx.x);
        u32x4 *z16 = reinterpret_cast<u32x4 *>(z + head);
        for (uint32_t x = threadIdx.x; x < n16; x += kMcGroupThreads) {
            const uint32_t o = head + 16 * x;
            uint32_t wd[4] = {0, 0, 0, 0};
            for (uint32_t row = o / nfile; row * nfile < o + 16; row++) {
                const uint32_t c = scand[row];
                const uint32_t at = row * nfile + c;
                if (c != 0xFFFFu && at >= o && at < o + 16) wd[(at - o) >> 2] |= 1u << (8 * ((at - o) & 3));
            }
            z16[x] = u32x4{wd[0], wd[1], wd[2], wd[3]};
        }
        if (tail + threadIdx.x < nz) z[tail + threadIdx.x] = (uint8_t)one_at(tail + threadIdx.x);
    }''')
old = '''            w.list[lh[c[p]] + rk[p]] = (uint32_t)i;
            hit[i * nfile + c[p]] = 1;'''
assert old in s
s = s.replace(old, '''            w.list[lh[c[p]] + rk[p]] = (uint32_t)i;''')
open('encode.hip', 'w').write(s)
print('ok fill')
