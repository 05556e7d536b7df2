# Diagnostic variant (scripts/build_variant.sh): the MayContain tests stage each filter's LDS part with streaming (slc) loads, so the bytes read past the LDS part stay in L2
s = open('encode.hip').read()
old = '''            (__attribute__((address_space(3))) void *)(lds + 16 * xw), 16, 0, 0);'''
assert s.count(old) == 1
s = s.replace(old, '''            (__attribute__((address_space(3))) void *)(lds + 16 * xw), 16, 0, 2);''')
open('encode.hip', 'w').write(s)
