# A/B variant: the all-tables hit matrix's zero rows (mc_classify_kernel) by non-temporal
# 16-byte stores (the matrix is written once here and touched again only at candidates).
s = open('encode.hip').read()
old = '''        for (uint64_t x = threadIdx.x; x < n16; x += kMcGroupThreads) z16[x] = make_uint4(0, 0, 0, 0);'''
assert old in s
s = s.replace(old, '''        for (uint64_t x = threadIdx.x; x < n16; x += kMcGroupThreads)
            __builtin_nontemporal_store(u32x4{0, 0, 0, 0}, reinterpret_cast<u32x4 *>(z16) + x);''')
open('encode.hip', 'w').write(s)
print('ok ntzero')
