# Diagnostic variant (scripts/build_variant.sh): 8 waves per SIMD for the data-region copy only (83 -> 56 VGPRs, no spills)
s = open('encode.hip').read()
a = "__global__ __launch_bounds__(256) void sst_vregion_runs_kernel"
assert a in s
s = s.replace(a, "__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void sst_vregion_runs_kernel")
open('encode.hip', 'w').write(s)
