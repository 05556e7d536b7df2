# A/B variant (on the source after the bit-read change): the level test's LDS copy of each
# filter 151 KiB instead of 144 (the scan's scratch row in the filter's LDS).
s = open('encode.hip').read()
old = '''    __shared__ uint32_t sg[kLvMaxWgs];      // its first slot in that workgroup
    __shared__ uint32_t part[kLvThreads];
    const uint32_t f = blockIdx.x, t = threadIdx.x;'''
assert old in s
s = s.replace(old, '''    __shared__ uint32_t sg[kLvMaxWgs];      // its first slot in that workgroup
    uint32_t *part = reinterpret_cast<uint32_t *>(fbytes);  // scan scratch, before the staging
    const uint32_t f = blockIdx.x, t = threadIdx.x;''')
old = '''    const uint64_t in_lds = stage_filter(src, F.nbits, fbytes, kMcLdsBytes, f, delta);
    __asm__ __volatile__("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint8_t *lb = fbytes + delta;
    while (q < total) {'''
assert old in s
s = s.replace(old, '''    const uint64_t in_lds = stage_filter(src, F.nbits, fbytes, kLvLdsBytes, f, delta);
    __asm__ __volatile__("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint8_t *lb = fbytes + delta;
    while (q < total) {''')
# every thread reads sb[nwg] (after the scan's last barrier) before any wave can start the
# staging: the early-return test reads total, then slot_of -- both before stage_filter;
# part[] is last read by `sb[nwg] = part[kLvThreads - 1]` before the barrier that precedes
# `total`, so the staging cannot overwrite a live part[] value.
old = '''constexpr uint32_t kLvMaxWgs = 1024;  // classify workgroups per pass (2M probes)'''
assert old in s
s = s.replace(old, old + '''
constexpr uint32_t kLvLdsBytes = 151 * 1024;  // the level test's filter bytes in LDS''')
old = '''            hipLaunchKernelGGL(lv_test_kernel, dim3(nfile), dim3(kLvThreads), kMcLdsBytes, s, d_img,'''
assert old in s
s = s.replace(old, '''            hipLaunchKernelGGL(lv_test_kernel, dim3(nfile), dim3(kLvThreads), kLvLdsBytes, s, d_img,''')
open('encode.hip', 'w').write(s)
print('ok lds2')
