# A/B variant: scripts/patch_lv_grid.py plus the filter's tail (the bytes past the LDS
# copy) warmed into the workgroup's L2 during the staging: one dword load per 128-byte
# line, waited for with the staging loads, so the probe loop's tail reads hit L2.
import os
os.environ['LV_PART'] = 'grid'
try:
    exec(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'patch_lv_pipe.py')).read())
except SystemExit:
    pass
s = open('encode.hip').read()
old = '''    const uint64_t in_lds = stage_filter(src, F.nbits, fbytes, kMcLdsBytes, f, delta);
    __asm__ __volatile__("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint8_t *lb = fbytes + delta;
    while (q < total) {'''
assert old in s
s = s.replace(old, '''    const uint64_t in_lds = stage_filter(src, F.nbits, fbytes, kMcLdsBytes, f, delta);
    {
        const uint64_t nb = 8 * (F.nbits / 64 + ((F.nbits & 63) != 0));
        for (uint64_t o = (in_lds & ~127ull) + 128ull * t; o < nb; o += 128ull * kLvThreads) {
            uint32_t v;
            const uint32_t *pw = reinterpret_cast<const uint32_t *>((uintptr_t)(src + o) & ~(uintptr_t)3);
            __asm__ __volatile__("global_load_dword %0, %1, off" : "=v"(v) : "v"(pw) : "memory");
        }
    }
    __asm__ __volatile__("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint8_t *lb = fbytes + delta;
    while (q < total) {''')
open('encode.hip', 'w').write(s)
print('ok tail')
