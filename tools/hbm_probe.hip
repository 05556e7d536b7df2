// hbm_probe.hip — calibration kernels for the roofline (tools only, never the
// product): achievable HBM read bandwidth on this box with (a) plain
// global_load_dwordx4 streaming, (b) buffer_load_dwordx4 ... lds in 1 KiB
// wave chunks (the decode kernel's load path), (c) a float4 copy.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void read_dwordx4(const u32x4 *in, uint64_t n16, uint32_t *sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
         i += (uint64_t)gridDim.x * blockDim.x) {
        u32x4 v = in[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;  // keeps the loads live
}

__global__ __launch_bounds__(256) void read_lds_dma(const uint8_t *in, uint64_t nbytes, uint32_t *sink) {
    __shared__ __attribute__((aligned(16))) uint32_t buf[4][1024];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nchunks = nbytes / 4096;
    uint32_t acc = 0;
    for (uint64_t c = (uint64_t)blockIdx.x * 4 + wave; c < nchunks; c += (uint64_t)gridDim.x * 4) {
        __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(in + c * 4096), 0, 4096, 0x00020000);
        for (int k = 0; k < 4; k++)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)&buf[wave][k * 256], 16, k * 1024 + lane * 16, 0, 0, 0);
        __asm__ __volatile__("s_waitcnt vmcnt(0)" ::: "memory");
        acc ^= buf[wave][lane];
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void copy_dwordx4(const u32x4 *in, u32x4 *out, uint64_t n16) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
         i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}

extern "C" int probe_read(const void *in, uint64_t nbytes, void *sink, int grid, void *stream) {
    hipLaunchKernelGGL(read_dwordx4, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4 *)in, nbytes / 16, (uint32_t *)sink);
    return (int)hipGetLastError();
}
extern "C" int probe_read_lds(const void *in, uint64_t nbytes, void *sink, int grid, void *stream) {
    hipLaunchKernelGGL(read_lds_dma, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (const uint8_t *)in, nbytes, (uint32_t *)sink);
    return (int)hipGetLastError();
}
extern "C" int probe_copy(const void *in, void *out, uint64_t nbytes, int grid, void *stream) {
    hipLaunchKernelGGL(copy_dwordx4, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4 *)in, (u32x4 *)out, nbytes / 16);
    return (int)hipGetLastError();
}
