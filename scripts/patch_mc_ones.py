# A/B variant (on the slot-grouped all-tables path): the rows zeroed early as now; after
# the searches every zero store is waited for (s_waitcnt vmcnt(0) before the barrier, so
# the workgroup's stores to one address stay ordered), then each candidate's thread writes
# its 1, and the test writes only the 0s of failed candidates.
s = open('encode.hip').read()
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
    // every zero store of this workgroup done before any of its 1s is issued
    __asm__ __volatile__("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (uint32_t p = 0; p < kMcGroupPer; p++) {
        if (cand[p] == kMcNone) continue;
        const uint64_t i = k_begin + (uint64_t)blockIdx.x * kMcGroupProbes + p * kMcGroupThreads + t;
        hit[i * nfile + cand[p]] = 1;
    }''')
old = '''        if (Matrix) may[(k_begin + id) * nfile + f] = (uint8_t)r;'''
assert old in s
s = s.replace(old, '''        if (Matrix) {
            if (!r) may[(k_begin + id) * nfile + f] = 0;  // classify wrote the 1
        }''')
open('encode.hip', 'w').write(s)
print('ok ones')
