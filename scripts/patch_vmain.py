# Diagnostic variant (scripts/build_variant.sh): the views build's data-region copy (its longest kernel) on the caller's stream, the keys / index regions / filters on the side stream (the join then rarely waits)
s = open('encode.hip').read()
old = '''    hipStream_t vs = vfork ? ctx->side : rs;  // the V region's stream'''
assert old in s
s = s.replace(old, '''    hipStream_t vs = vfork ? s : rs;  // the V region's stream
    if (vfork) rs = ctx->side;''')
old = '''        hipLaunchKernelGGL(bloom_or_kernel, dim3((nfile + 7) / 8 * 16), dim3(1024), (size_t)(osb / 8), s,
                           bo, a);'''
assert old in s
s = s.replace(old, '''        hipLaunchKernelGGL(bloom_or_kernel, dim3((nfile + 7) / 8 * 16), dim3(1024), (size_t)(osb / 8), rs,
                           bo, a);''')
open('encode.hip', 'w').write(s)
