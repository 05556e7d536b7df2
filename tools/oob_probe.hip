// Probe: how the raw-buffer range check treats a 16-byte load (to VGPRs and
// LDS-DMA) that straddles num_records.  Prints, per case, the four dwords a
// lane received; dwords of the source are 0x1000 + index.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void probe(const uint32_t *src, uint32_t bytes, uint32_t *out) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[64 * 4];
    const uint32_t lane = threadIdx.x;
    rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(src), (short)0, (int)bytes,
                                                 0x00020000);
    for (uint32_t i = lane; i < 256; i += 64) lds[i] = 0xdeadbeef;
    __syncthreads();
    const uint32_t off = 4 * lane;  // lane l reads bytes [4l, 4l + 16)
    u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)&lds[0], 16,
                                             off, 0, 0, 0);
    __asm__ __volatile__("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int k = 0; k < 4; k++) {
        out[8 * lane + k] = v[k];
        out[8 * lane + 4 + k] = lds[4 * lane + k];
    }
}

int main() {
    uint32_t h[128];
    for (int i = 0; i < 128; i++) h[i] = 0x1000 + i;
    uint32_t *d, *o;
    hipMalloc(&d, sizeof h);
    hipMalloc(&o, 64 * 8 * 4);
    hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
    const uint32_t bytes = 40;  // dwords 0..9 in range
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, bytes, o);
    uint32_t r[64 * 8];
    if (hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    for (int l = 5; l < 11; l++)
        printf("lane %d (bytes %d..%d, range %u): vgpr %x %x %x %x  lds %x %x %x %x\n", l, 4 * l,
               4 * l + 16, bytes, r[8 * l], r[8 * l + 1], r[8 * l + 2], r[8 * l + 3], r[8 * l + 4],
               r[8 * l + 5], r[8 * l + 6], r[8 * l + 7]);
    return 0;
}
