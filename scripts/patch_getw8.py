# Diagnostic variant (scripts/build_variant.sh): 8 waves per SIMD for the Get kernel (72 -> 64 VGPRs, 36 B scratch)
s = open('encode.hip').read()
a = "__global__ __launch_bounds__(256) void level_get_kernel(GetArgs a) {"
assert a in s
s = s.replace(a, "__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void level_get_kernel(GetArgs a) {")
open('encode.hip', 'w').write(s)
