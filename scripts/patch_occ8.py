# Diagnostic variant (scripts/build_variant.sh): 8 waves per SIMD for the data-region copy (83 -> 56 VGPRs) and the IDX-only region writer (71 -> 64 VGPRs), no spills
s = open('encode.hip').read()
a = "__global__ __launch_bounds__(256) void sst_vregion_runs_kernel"
assert a in s
s = s.replace(a, "__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void sst_vregion_runs_kernel")
b = "template <bool WithV>\n__global__ __launch_bounds__(kRegWaves *kWave) void sst_regions_kernel(SstArgs a) {"
assert b in s
s = s.replace(b, "template <bool WithV>\n__global__ __launch_bounds__(kRegWaves *kWave) __attribute__((amdgpu_waves_per_eu(WithV ? 4 : 8))) void sst_regions_kernel(SstArgs a) {")
open('encode.hip', 'w').write(s)
