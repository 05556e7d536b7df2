// api.hip — context management of the C ABI (include/lsm_gpu.h).
#include <stdlib.h>
#include <string.h>

#include "common.h"

extern "C" int lsm_abi_version(void) { return LSM_ABI_VERSION; }
extern "C" int lsm_input_slack(void) { return LSM_INPUT_SLACK; }
#ifndef LSM_BUILD_ID
#define LSM_BUILD_ID "unknown"
#endif
// hash of the sources this library was compiled from (go-lsm_amd/build_id.py)
extern "C" const char *lsm_build_id(void) { return LSM_BUILD_ID; }
#ifndef LSM_BUILD_FLAGS
#define LSM_BUILD_FLAGS ""
#endif
// "HIPCC|ARCH|HIPFLAGS" the library was compiled with (part of the build id)
extern "C" const char *lsm_build_flags(void) { return LSM_BUILD_FLAGS; }

extern "C" int lsm_ctx_create(int device, lsm_ctx **out) {
    if (!out) return LSM_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return LSM_ENODEV;
    if (device < 0 || device >= n) return LSM_ENODEV;
    hipDeviceProp_t prop;
    LSM_HIP_CHECK(hipGetDeviceProperties(&prop, device));
    // The kernels are built for gfx950 only (CDNA4, MI355X).
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return LSM_ENODEV;
    lsm_ctx *c = static_cast<lsm_ctx *>(calloc(1, sizeof(lsm_ctx)));
    if (!c) return LSM_ENOMEM;
    c->device = device;
    c->num_cus = prop.multiProcessorCount;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->join, hipEventDisableTiming);
    if (e == hipSuccess) e = hipHostMalloc(&c->host_rb, kHostReadback, hipHostMallocDefault);
    if (e != hipSuccess) {
        lsm_ctx_destroy(c);
        return -(1000 + (int)e);
    }
    *out = c;
    return 0;
}

extern "C" int lsm_ctx_destroy(lsm_ctx *ctx) {
    if (!ctx) return 0;
    if (hipSetDevice(ctx->device) == hipSuccess) {
        if (ctx->join) (void)hipEventDestroy(ctx->join);
        if (ctx->fork) (void)hipEventDestroy(ctx->fork);
        if (ctx->side) (void)hipStreamDestroy(ctx->side);
        if (ctx->host_rb) (void)hipHostFree(ctx->host_rb);
        if (ctx->host_big) (void)hipHostFree(ctx->host_big);
    }
    free(ctx);
    return 0;
}

extern "C" int lsm_ctx_num_cus(const lsm_ctx *ctx) { return ctx ? ctx->num_cus : 0; }

static int bind(lsm_ctx *ctx) {
    if (!ctx) return LSM_EINVAL;
    LSM_HIP_CHECK(hipSetDevice(ctx->device));
    return 0;
}

extern "C" int lsm_dev_alloc(lsm_ctx *ctx, size_t bytes, void **out) {
    if (!out) return LSM_EINVAL;
    *out = nullptr;
    int rc = bind(ctx);
    if (rc) return rc;
    size_t n = ((bytes + 15) & ~(size_t)15) + LSM_INPUT_SLACK;  // include/lsm_gpu.h
    LSM_HIP_CHECK(hipMalloc(out, n));
    return 0;
}

extern "C" int lsm_dev_free(lsm_ctx *ctx, void *p) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (p) LSM_HIP_CHECK(hipFree(p));
    return 0;
}

extern "C" int lsm_host_alloc_pinned(lsm_ctx *ctx, size_t bytes, void **out) {
    if (!out) return LSM_EINVAL;
    *out = nullptr;
    int rc = bind(ctx);
    if (rc) return rc;
    LSM_HIP_CHECK(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
    return 0;
}

extern "C" int lsm_host_free_pinned(lsm_ctx *ctx, void *p) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (p) LSM_HIP_CHECK(hipHostFree(p));
    return 0;
}

extern "C" int lsm_memcpy_h2d(lsm_ctx *ctx, void *d_dst, const void *h_src, size_t bytes,
                              void *stream) {
    if (!ctx || (bytes && (!d_dst || !h_src))) return LSM_EINVAL;
    if (!bytes) return 0;
    LSM_HIP_CHECK(hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice,
                                 static_cast<hipStream_t>(stream)));
    return 0;
}

extern "C" int lsm_memcpy_d2h(lsm_ctx *ctx, void *h_dst, const void *d_src, size_t bytes,
                              void *stream) {
    if (!ctx || (bytes && (!d_src || !h_dst))) return LSM_EINVAL;
    if (!bytes) return 0;
    LSM_HIP_CHECK(hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost,
                                 static_cast<hipStream_t>(stream)));
    return 0;
}

extern "C" int lsm_memset_dev(lsm_ctx *ctx, void *d_dst, int value, size_t bytes, void *stream) {
    if (!ctx || (bytes && !d_dst)) return LSM_EINVAL;
    if (!bytes) return 0;
    LSM_HIP_CHECK(hipMemsetAsync(d_dst, value, bytes, static_cast<hipStream_t>(stream)));
    return 0;
}

extern "C" int lsm_stream_create(lsm_ctx *ctx, void **out) {
    if (!out) return LSM_EINVAL;
    int rc = bind(ctx);
    if (rc) return rc;
    hipStream_t s;
    LSM_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *out = s;
    return 0;
}

extern "C" int lsm_stream_destroy(lsm_ctx *ctx, void *stream) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (stream) LSM_HIP_CHECK(hipStreamDestroy(static_cast<hipStream_t>(stream)));
    return 0;
}

extern "C" int lsm_stream_sync(lsm_ctx *ctx, void *stream) {
    if (!ctx) return LSM_EINVAL;
    LSM_HIP_CHECK(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    return 0;
}
