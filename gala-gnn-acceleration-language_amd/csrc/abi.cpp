// C-ABI bookkeeping of libgala_hip.so: status strings, argument validation and the
// segment table (column-tiled graphs, src/ops/tiling.h:222-283).
#include <hip/hip_runtime.h>

#include "gala_internal.h"

namespace gala {

static thread_local int g_last_hip_error = 0;

void set_last_hip_error(int e) { g_last_hip_error = e; }

int launch_status() {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_hip_error((int)e);
        return GALA_ERR_HIP;
    }
    return GALA_OK;
}

int check_csr(const gala_csr_t *A) {
    if (!A) return GALA_ERR_INVALID_ARG;
    if (A->n_rows < 0 || A->n_cols < 0 || A->nnz < 0 || A->n_seg < 1) return GALA_ERR_INVALID_ARG;
    if (A->n_rows > 0 && !A->rowptr) return GALA_ERR_INVALID_ARG;
    if (A->nnz > 0 && !A->col) return GALA_ERR_INVALID_ARG;
    if (A->n_seg > 1 && !A->seg_bounds) return GALA_ERR_INVALID_ARG;
    if (A->val && A->val_heads < 1) return GALA_ERR_INVALID_ARG;
    if (A->nnz > INT32_MAX || A->n_rows >= INT32_MAX || A->n_cols > INT32_MAX)
        return GALA_ERR_UNSUPPORTED;  // int32 index contract of the reference
    return GALA_OK;
}

int fill_segments(const gala_csr_t *A, int32_t first, SegTable *t) {
    const int32_t n = A->n_seg - first;
    t->n = n < kMaxSegPerLaunch ? n : kMaxSegPerLaunch;
    for (int32_t i = 0; i < t->n; ++i) {
        const int32_t s = first + i;
        t->rp[i] = s;
        if (A->n_seg == 1) {
            t->base[i] = 0;
        } else {
            const int32_t b0 = A->seg_bounds[2 * s], b1 = A->seg_bounds[2 * s + 1];
            if (b0 < 0 || b1 < b0 || b1 > A->nnz) return GALA_ERR_GRAPH;
            t->base[i] = b0;
        }
    }
    return GALA_OK;
}

}  // namespace gala

extern "C" int gala_abi_version(void) { return GALA_ABI_VERSION; }

extern "C" int gala_last_hip_error(void) { return gala::g_last_hip_error; }

extern "C" const char *gala_status_string(int status) {
    switch (status) {
        case GALA_OK: return "GALA_OK";
        case GALA_ERR_INVALID_ARG: return "GALA_ERR_INVALID_ARG";
        case GALA_ERR_UNSUPPORTED: return "GALA_ERR_UNSUPPORTED";
        case GALA_ERR_HIP: return "GALA_ERR_HIP";
        case GALA_ERR_GRAPH: return "GALA_ERR_GRAPH";
        default: return "GALA_ERR_UNKNOWN";
    }
}
