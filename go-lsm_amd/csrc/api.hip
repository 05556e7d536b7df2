// api.hip — context management of the C ABI (include/lsm_gpu.h).
#include <stdlib.h>
#include <string.h>

#include "common.h"

struct lsm_ctx {
    int device;
    int num_cus;
};

extern "C" int lsm_abi_version(void) { return LSM_ABI_VERSION; }

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
    *out = c;
    return 0;
}

extern "C" int lsm_ctx_destroy(lsm_ctx *ctx) {
    free(ctx);
    return 0;
}

extern "C" int lsm_ctx_num_cus(const lsm_ctx *ctx) { return ctx ? ctx->num_cus : 0; }
