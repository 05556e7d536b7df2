# Diagnostic variant (scripts/build_variant.sh): wal_seg_lanes_kernel with per-section clock64() stamps;
# the last wave of each launch prints the mean cycles per wave of each section (never the product).
s = open('decode.hip').read()
k = '__global__ __launch_bounds__(64) void wal_seg_lanes_kernel(WalArgs a) {'
assert k in s
s = s.replace(k, '''__device__ unsigned long long g_walt[12];
__device__ unsigned int g_waln;
__device__ __forceinline__ void walt_add(int i, uint64_t d) {
    if (lane_id() == 0) atomicAdd(&g_walt[i], (unsigned long long)d);
}
''' + k + '''
    uint64_t T0 = clock64(), Tp = T0;
    auto stamp = [&](int i) { const uint64_t t = clock64(); walt_add(i, t - Tp); Tp = t; };''')
old = '''    uint32_t g = start, g1 = 0xFFFFFFFFu;  // entries of phase 0 and phase 1'''
assert old in s
s = s.replace(old, '''    stamp(0);  // staging
''' + old)
old = '''    const uint32_t E = start + kWalSeg < len ? start + kWalSeg : len;
    // 1. shares'''
assert old in s
s = s.replace(old, '''    stamp(1);  // the segment guess
''' + old)
old = '''    // 2. + 3. per phase: stitch from the entry, then write the accepted chains'''
assert old in s
s = s.replace(old, '''    stamp(2);  // first_plausible + chase2
''' + old)
old = '''        uint32_t tot;
        const uint32_t pre = wave_excl_scan(acc_cnt, &tot);'''
assert old in s
s = s.replace(old, '''        stamp(3 + 2 * ph);  // stitch
''' + old)
old = '''        if (lane == 0) a.seg[q] = WalSeg{gp, e, total, status};
    }
}'''
assert old in s
s = s.replace(old, '''        if (lane == 0) a.seg[q] = WalSeg{gp, e, total, status};
        stamp(4 + 2 * ph);  // scratch writes
    }
    walt_add(7, clock64() - T0);
    walt_add(8, 1);
    if (lane_id() == 0) {
        __threadfence();
        const unsigned int n = atomicAdd(&g_waln, 1u) + 1;
        if (n == gridDim.x * gridDim.y) {
            const double w = (double)atomicAdd(&g_walt[8], 0ull);
            printf("WALT waves %.0f stage %.0f guess %.0f shares %.0f stitch0 %.0f write0 %.0f stitch1 %.0f write1 %.0f total %.0f\\n", w,
                   atomicAdd(&g_walt[0], 0ull) / w, atomicAdd(&g_walt[1], 0ull) / w, atomicAdd(&g_walt[2], 0ull) / w,
                   atomicAdd(&g_walt[3], 0ull) / w, atomicAdd(&g_walt[4], 0ull) / w, atomicAdd(&g_walt[5], 0ull) / w,
                   atomicAdd(&g_walt[6], 0ull) / w, atomicAdd(&g_walt[7], 0ull) / w);
            for (int i = 0; i < 12; i++) atomicExch(&g_walt[i], 0ull);
            atomicExch(&g_waln, 0u);
        }
    }
}''')
old = '''        if (lane == 0) a.seg[q0] = a.seg[q0 + 1] = WalSeg{0xFFFFFFFFu, 0xFFFFFFFFu, 0, 0};
        return;
    }'''
assert old in s
s = s.replace(old, '''        if (lane == 0) a.seg[q0] = a.seg[q0 + 1] = WalSeg{0xFFFFFFFFu, 0xFFFFFFFFu, 0, 0};
        if (lane == 0) { __threadfence(); atomicAdd(&g_waln, 1u); }  // (a launch's last wave is a working one)
        return;
    }''')
open('decode.hip', 'w').write(s)
print('ok')
