# Diagnostic variant (scripts/build_variant.sh): the WAL segment kernel's scratch entries collected in LDS and stored by 16-byte coalesced rows (2 KiB buffer per wave; direct stores past it)
import sys
NB = int(sys.argv[1]) if len(sys.argv) > 1 else 512
s = open('decode.hip').read()
old = '''    __shared__ __attribute__((aligned(16))) uint32_t stage[STAGE / 4 + 4];'''
assert old in s
s = s.replace(old, old + '''
    __shared__ __attribute__((aligned(16))) uint32_t sent[%d];  // a phase's entries, stored by rows''' % NB)
old = '''        uint32_t tot;
        const uint32_t pre = wave_excl_scan(acc_cnt, &tot);
        if (acc_cnt) {
            uint32_t *dst = reinterpret_cast<uint32_t *>(a.scratch + q * kWalSegSlots) + pre;
            uint32_t p = acc_entry;
            for (uint32_t i = 0; i < acc_cnt; i++) {
                uint32_t kl = 0, vl = 0;
                L.record(p, kl, vl);
                dst[i] = (p - start) | (kl < kWalKlEsc ? kl : kWalKlEsc) << kWalPosBits;
                p += 8 + kl + vl;
            }
        }'''
assert old in s
s = s.replace(old, '''        uint32_t tot;
        const uint32_t pre = wave_excl_scan(acc_cnt, &tot);
        uint32_t *gdst = reinterpret_cast<uint32_t *>(a.scratch + q * kWalSegSlots);
        {
            uint32_t p = acc_entry;
            for (uint32_t i = 0; i < acc_cnt; i++) {
                uint32_t kl = 0, vl = 0;
                L.record(p, kl, vl);
                const uint32_t e = (p - start) | (kl < kWalKlEsc ? kl : kWalKlEsc) << kWalPosBits;
                if (pre + i < %d) sent[pre + i] = e;
                else gdst[pre + i] = e;
                p += 8 + kl + vl;
            }
        }
        __builtin_amdgcn_wave_barrier();
        __asm__ __volatile__("" ::: "memory");
        {
            const uint32_t nb = uni(tot) < %d ? uni(tot) : %d;
            for (uint32_t t = 4 * lane; t < nb; t += 4 * kWave)
                *reinterpret_cast<u32x4 *>(gdst + t) = *reinterpret_cast<const u32x4 *>(&sent[t]);
        }
        __builtin_amdgcn_wave_barrier();
        __asm__ __volatile__("" ::: "memory");''' % (NB, NB, NB))
open('decode.hip', 'w').write(s)
print('ok', NB)
