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


// copy variants: U float4s in flight per thread, optional nontemporal stores /
// loads; and one float4 per thread over a grid covering the buffer
template <int U, bool NTS, bool NTL>
__global__ __launch_bounds__(256) void copy_var(const u32x4 *in, u32x4 *out, uint64_t n16) {
    const uint64_t st = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += U * st) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++)
            if (i + u * st < n16) v[u] = NTL ? __builtin_nontemporal_load(&in[i + u * st]) : in[i + u * st];
#pragma unroll
        for (int u = 0; u < U; u++)
            if (i + u * st < n16) {
                if (NTS) __builtin_nontemporal_store(v[u], &out[i + u * st]);
                else out[i + u * st] = v[u];
            }
    }
}
__global__ __launch_bounds__(256) void copy_flat(const u32x4 *in, u32x4 *out, uint64_t n16) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n16) out[i] = in[i];
}
extern "C" int probe_copy_var(const void *in, void *out, uint64_t nbytes, int grid, int kind, void *stream) {
    const u32x4 *a = (const u32x4 *)in;
    u32x4 *b = (u32x4 *)out;
    hipStream_t s = (hipStream_t)stream;
    const uint64_t n16 = nbytes / 16;
    switch (kind) {
    case 0: hipLaunchKernelGGL((copy_var<4, false, false>), dim3(grid), dim3(256), 0, s, a, b, n16); break;
    case 1: hipLaunchKernelGGL((copy_var<4, true, false>), dim3(grid), dim3(256), 0, s, a, b, n16); break;
    case 2: hipLaunchKernelGGL((copy_var<4, true, true>), dim3(grid), dim3(256), 0, s, a, b, n16); break;
    case 3: hipLaunchKernelGGL((copy_var<1, true, false>), dim3(grid), dim3(256), 0, s, a, b, n16); break;
    default: hipLaunchKernelGGL(copy_flat, dim3((uint32_t)((n16 + 255) / 256)), dim3(256), 0, s, a, b, n16); break;
    }
    return (int)hipGetLastError();
}

// ---- block-shaped probes (decode4k's memory pattern without the parse) ------
// Each wave stages one 4 KiB block into LDS by four 1 KiB LDS-DMAs, waits,
// and writes 33 x 16 B descriptors (the DESC output of a 33-record block).
template <int WPG, bool META, int LAUX = 0, bool NTST = false>
__global__ __launch_bounds__(64 * WPG) void blocks_dma(const uint8_t *in, const uint64_t *off,
                                                      const uint32_t *len, uint32_t nblk, u32x4 *out) {
    __shared__ __attribute__((aligned(16))) uint32_t buf[WPG][1024];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t b = blockIdx.x * WPG + wave;
    if (b >= nblk) return;
    uint64_t o = (uint64_t)b * 4096;
    uint32_t n = 4096;
    if (META) {
        o = __builtin_amdgcn_readfirstlane((uint32_t)off[b]) |
            (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(off[b] >> 32)) << 32;
        n = __builtin_amdgcn_readfirstlane(len[b]);
    }
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(in + o), 0, n, 0x00020000);
    for (int k = 0; k < 4; k++)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)&buf[wave][k * 256], 16, k * 1024 + lane * 16, 0, 0, LAUX);
    __asm__ __volatile__("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t v = buf[wave][lane * 31 % 1024];
    if (lane < 33) {
        u32x4 d = {v, (uint32_t)o, lane, 100};
        if (NTST) __builtin_nontemporal_store(d, &out[(uint64_t)b * 33 + lane]);
        else out[(uint64_t)b * 33 + lane] = d;
    }
}

// Persistent, double-buffered: wave w walks blocks w, w+W, ...; block k+1's
// DMAs are in flight while block k is "processed".
template <int WPG>
__global__ __launch_bounds__(64 * WPG) void blocks_dma_db(const uint8_t *in, uint32_t nblk, u32x4 *out) {
    __shared__ __attribute__((aligned(16))) uint32_t buf[WPG][2][1024];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t W = gridDim.x * WPG;
    uint32_t b = blockIdx.x * WPG + wave;
    if (b >= nblk) return;
    auto stage = [&](uint32_t bb, uint32_t slot) {
        __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(in + (uint64_t)bb * 4096), 0, 4096, 0x00020000);
        for (int k = 0; k < 4; k++)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)&buf[wave][slot][k * 256], 16, k * 1024 + lane * 16, 0, 0, 0);
    };
    stage(b, 0);
    for (uint32_t k = 0;; k++) {
        const uint32_t nb = b + W;
        if (nb < nblk) {
            stage(nb, (k + 1) & 1);
            __asm__ __volatile__("s_waitcnt vmcnt(4)" ::: "memory");
        } else {
            __asm__ __volatile__("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const uint32_t v = buf[wave][k & 1][lane * 31 % 1024];
        if (lane < 33) {
            u32x4 d = {v, b, lane, 100};
            out[(uint64_t)b * 33 + lane] = d;
        }
        if (nb >= nblk) break;
        b = nb;
    }
}

extern "C" int probe_blocks(int mode, const void *in, const uint64_t *off, const uint32_t *len,
                            uint32_t nblk, void *out, int grid, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    u32x4 *o = (u32x4 *)out;
    const uint8_t *i = (const uint8_t *)in;
    switch (mode) {
    case 0: hipLaunchKernelGGL((blocks_dma<4, false>), dim3((nblk + 3) / 4), dim3(256), 0, s, i, off, len, nblk, o); break;
    case 1: hipLaunchKernelGGL((blocks_dma<4, true>), dim3((nblk + 3) / 4), dim3(256), 0, s, i, off, len, nblk, o); break;
    case 2: hipLaunchKernelGGL((blocks_dma<1, true>), dim3(nblk), dim3(64), 0, s, i, off, len, nblk, o); break;
    case 3: hipLaunchKernelGGL((blocks_dma<8, true>), dim3((nblk + 7) / 8), dim3(512), 0, s, i, off, len, nblk, o); break;
    case 4: hipLaunchKernelGGL((blocks_dma_db<4>), dim3(grid), dim3(256), 0, s, i, nblk, o); break;
    case 5: hipLaunchKernelGGL((blocks_dma_db<1>), dim3(grid), dim3(64), 0, s, i, nblk, o); break;
    case 6: hipLaunchKernelGGL((blocks_dma<4, true, 0, true>), dim3((nblk + 3) / 4), dim3(256), 0, s, i, off, len, nblk, o); break;
    case 7: hipLaunchKernelGGL((blocks_dma<4, true, 2, false>), dim3((nblk + 3) / 4), dim3(256), 0, s, i, off, len, nblk, o); break;
    case 8: hipLaunchKernelGGL((blocks_dma<4, true, 2, true>), dim3((nblk + 3) / 4), dim3(256), 0, s, i, off, len, nblk, o); break;
    case 9: hipLaunchKernelGGL((blocks_dma<4, true, 1, false>), dim3((nblk + 3) / 4), dim3(256), 0, s, i, off, len, nblk, o); break;
    case 10: hipLaunchKernelGGL((blocks_dma<4, true, 17, true>), dim3((nblk + 3) / 4), dim3(256), 0, s, i, off, len, nblk, o); break;
    default: return -1;
    }
    return (int)hipGetLastError();
}

// ---- long-block streaming probe (the large-block decode's memory pattern) --
// Persistent one-wave workgroups; wave w streams blocks w, w+W, ... of
// `blk` bytes each through an NCH x 1 KiB LDS ring: consuming chunk c waits
// (counted vmcnt) for chunk c only and tops the ring up to c + NCH - 1.
template <int N>
__device__ __forceinline__ void probe_wait(uint32_t k) {
#define PW(i) case i: __asm__ __volatile__("s_waitcnt vmcnt(" #i ")" ::: "memory"); break;
    switch (k < N ? k : N - 1) {
    PW(0) PW(1) PW(2) PW(3) PW(4) PW(5) PW(6) PW(7) PW(8) PW(9) PW(10) PW(11) PW(12) PW(13) PW(14)
    default: __asm__ __volatile__("s_waitcnt vmcnt(15)" ::: "memory"); break;
    }
#undef PW
}

template <int NCH, int AUX>
__global__ __launch_bounds__(64) void stream_ring(const uint8_t *in, uint32_t nblk, uint32_t blk,
                                                  uint32_t *sink) {
    __shared__ __attribute__((aligned(16))) uint32_t ring[NCH * 256];
    const uint32_t lane = threadIdx.x & 63;
    uint32_t acc = 0;
    for (uint32_t b = blockIdx.x; b < nblk; b += gridDim.x) {
        __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(in + (uint64_t)b * blk), 0, blk, 0x00020000);
        const uint32_t nch = blk / 1024;
        uint32_t hi = 0;
        for (uint32_t c = 0; c < nch; c++) {
            uint32_t last = c + NCH < nch ? c + NCH : nch;
            for (; hi < last; hi++)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)&ring[(hi % NCH) * 256], 16, hi * 1024 + lane * 16, 0, 0, AUX);
            probe_wait<NCH>(hi - c - 1);
            acc ^= ring[(c % NCH) * 256 + lane * 4];
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

extern "C" int probe_stream(int nch, const void *in, uint32_t nblk, uint32_t blk, void *sink,
                            int grid, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    const uint8_t *i = (const uint8_t *)in;
    uint32_t *k = (uint32_t *)sink;
    switch (nch) {
    case 2: hipLaunchKernelGGL((stream_ring<2, 2>), dim3(grid), dim3(64), 0, s, i, nblk, blk, k); break;
    case 4: hipLaunchKernelGGL((stream_ring<4, 2>), dim3(grid), dim3(64), 0, s, i, nblk, blk, k); break;
    case 8: hipLaunchKernelGGL((stream_ring<8, 2>), dim3(grid), dim3(64), 0, s, i, nblk, blk, k); break;
    case 16: hipLaunchKernelGGL((stream_ring<16, 2>), dim3(grid), dim3(64), 0, s, i, nblk, blk, k); break;
    case 116: hipLaunchKernelGGL((stream_ring<16, 0>), dim3(grid), dim3(64), 0, s, i, nblk, blk, k); break;
    case 108: hipLaunchKernelGGL((stream_ring<8, 0>), dim3(grid), dim3(64), 0, s, i, nblk, blk, k); break;
    default: return -1;
    }
    return (int)hipGetLastError();
}

// Buffer range-check semantics: 64 lanes store 4 bytes each at voffset 4*lane,
// soffset `so`, instruction offset 0, through a descriptor of `nrec` bytes;
// which dwords land tells whether soffset counts in the check.
__global__ void range_store(uint32_t *out, uint32_t nrec, uint32_t so) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out, 0, nrec, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(1u + threadIdx.x, r, 4 * threadIdx.x, so, 0);
}
extern "C" int probe_range(void *out, uint32_t nrec, uint32_t so, void *stream) {
    hipLaunchKernelGGL(range_store, dim3(1), dim3(64), 0, (hipStream_t)stream, (uint32_t *)out, nrec, so);
    return (int)hipGetLastError();
}
