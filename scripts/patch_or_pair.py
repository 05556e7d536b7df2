# Diagnostic variant (scripts/build_variant.sh): bloom_or_kernel with the two slices of a filter dealt to one XCD at the same time
s = open('encode.hip').read()
old = '''    extern __shared__ __attribute__((aligned(16))) uint32_t lds_bits[];
    const uint32_t f = blockIdx.x, sl = blockIdx.y;'''
new = '''    extern __shared__ __attribute__((aligned(16))) uint32_t lds_bits[];
    // workgroups b and b + 8 share an XCD (blocks are dealt round-robin over
    // the 8 XCDs, the guide's observed placement; speed only): the two
    // slices of filter f are blocks 16 (f / 8) + f % 8 and that + 8, so they
    // run side by side on one XCD and the second read of the filter's hash
    // records is served by that XCD's L2
    const uint32_t b = blockIdx.x, f = (b / 16) * 8 + b % 8, sl = (b / 8) % 2;
    if (f >= a.nfiles) return;'''
assert old in s; s = s.replace(old, new)
old = '''        hipLaunchKernelGGL(bloom_or_kernel, dim3(nfile, (uint32_t)((m + osb - 1) / osb)), dim3(1024),
                           (size_t)(osb / 8), s, bo, a);'''
new = '''        bo.nfiles = nfile;
        hipLaunchKernelGGL(bloom_or_kernel, dim3((nfile + 7) / 8 * 16), dim3(1024), (size_t)(osb / 8), s,
                           bo, a);'''
assert old in s; s = s.replace(old, new)
old = '''    uint32_t split;     // slice 0 = bits [0, split), slice 1 = [split, m)
    uint64_t nwords;'''
new = '''    uint32_t split;     // slice 0 = bits [0, split), slice 1 = [split, m)
    uint32_t nfiles;
    uint64_t nwords;'''
assert old in s; s = s.replace(old, new)
open('encode.hip', 'w').write(s)
