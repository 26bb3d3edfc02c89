// libgala_cpu.so — host-CPU backend of the operator set (include/gala_cpu.h).
//
// The reference has no CPU code generator (src/codegen/cpu.h:1-7); its only CPU
// aggregation is the gSpMM/wsumAgg pair used by its host-side tiling code
// (src/ops/aggregators.h:12-127).  This file gives every entry point of gala_hip.h a CPU
// counterpart with the same signature, validation and status codes, so a generated
// program runs unchanged on the host cores when it places its tensors there (config 1 of
// BASELINE.json: Cora GCN on CPU).  Rows are distributed over OpenMP threads; inside a
// row the edges are accumulated in CSR order with the reference's rounding steps
// (compiled with -ffp-contract=off; fmaf exactly where nvcc contracts the emitted
// kernels' `a + b*c`), which makes SpMM, degree, SDDVV, row-scale and row-broadcast
// bit-identical to libgala_hip.so.
#include <math.h>
#include <omp.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/gala_cpu.h"

namespace {

int check_csr(const gala_csr_t *A) {
    if (!A) return GALA_ERR_INVALID_ARG;
    if (A->n_rows < 0 || A->n_cols < 0 || A->nnz < 0 || A->n_seg < 1) return GALA_ERR_INVALID_ARG;
    if (A->n_rows > 0 && !A->rowptr) return GALA_ERR_INVALID_ARG;
    if (A->nnz > 0 && !A->col) return GALA_ERR_INVALID_ARG;
    if (A->n_seg > 1 && !A->seg_bounds) return GALA_ERR_INVALID_ARG;
    if (A->val && A->val_heads < 1) return GALA_ERR_INVALID_ARG;
    if (A->nnz > INT32_MAX || A->n_rows >= INT32_MAX || A->n_cols > INT32_MAX)
        return GALA_ERR_UNSUPPORTED;
    for (int32_t s = 0; A->n_seg > 1 && s < A->n_seg; ++s) {
        const int32_t b0 = A->seg_bounds[2 * s], b1 = A->seg_bounds[2 * s + 1];
        if (b0 < 0 || b1 < b0 || b1 > A->nnz) return GALA_ERR_GRAPH;
    }
    return GALA_OK;
}

// edges [e0, e1) of row r in segment s (relative offsets + segment base, tiling.h:222-283)
inline void row_range(const gala_csr_t *A, int32_t s, int64_t r, int64_t &e0, int64_t &e1) {
    const int32_t *rp = A->rowptr + (int64_t)s * (A->n_rows + 1);
    const int64_t base = A->n_seg == 1 ? 0 : A->seg_bounds[2 * s];
    e0 = base + rp[r];
    e1 = base + rp[r + 1];
}

inline float ref_exp(float s) {
    const float p = expf(s);  // torch::exp then clamp(0, 1e12) (common.h:760-761)
    return p > 1e12f ? 1e12f : p;
}

constexpr int64_t kRowChunk = 256;  // rows per OpenMP work item

}  // namespace

extern "C" int gala_cpu_spmm_f32(const gala_csr_t *A, const float *X, int64_t ldx, float *Y,
                                 int64_t ldy, int32_t F, const float *src_scale,
                                 const float *dst_scale, int32_t flags, int32_t nsamp,
                                 int32_t ra, int32_t rb, void *stream) {
    return gala_cpu_spmm_ex_f32(A, X, ldx, Y, ldy, F, src_scale, dst_scale, flags, nsamp, ra, rb, nullptr, stream);
}

// torch.relu as its GPU kernel computes it (the HIP backend's relu_t): t > 0 ? t : +0, NaN passes
static inline float relu_t(float t) { return (t > 0.0f || t != t) ? t : 0.0f; }

// (every row is one sequential pass here: GALA_SPMM_HUB_CHUNKED is accepted and gives the
// REF-order result, which is within that mode's tolerance)
extern "C" int gala_cpu_spmm_ex_f32(const gala_csr_t *A, const float *X, int64_t ldx, float *Y,
                                    int64_t ldy, int32_t F, const float *src_scale,
                                    const float *dst_scale, int32_t flags, int32_t nsamp,
                                    int32_t ra, int32_t rb, const gala_spmm_epilogue_t *epi, void *) {
    int st = check_csr(A);
    if (st) return st;
    if (F < 0 || ldx < F || ldy < F ||
        (flags & ~(GALA_SPMM_ACCUM | GALA_SPMM_SAMPLE | GALA_SPMM_EXACT | GALA_SPMM_HUB_CHUNKED)) ||
        ((flags & GALA_SPMM_EXACT) && (flags & GALA_SPMM_HUB_CHUNKED)))
        return GALA_ERR_INVALID_ARG;
    const bool dst_deg = epi && epi->dst_deg_rsqrt;
    float *Y2 = epi ? epi->Y2 : nullptr;
    const int64_t ldy2 = Y2 ? epi->ldy2 : 0;
    const float *y2s = Y2 ? epi->y2_scale : nullptr;
    if (dst_deg && (dst_scale || A->n_seg != 1 || A->val || (flags & GALA_SPMM_SAMPLE))) return GALA_ERR_UNSUPPORTED;
    if (Y2 && ldy2 < F) return GALA_ERR_INVALID_ARG;
    const bool relu_pro = epi && epi->src_relu;
    const float *src_act = relu_pro ? epi->src_act : nullptr;
    const float *relu_x = epi ? epi->relu_x : nullptr;
    const int64_t ldrx = relu_x ? epi->ldrx : 0;
    const float *relu_act = relu_x ? epi->relu_act : nullptr;
    if (epi && epi->src_act && !relu_pro) return GALA_ERR_INVALID_ARG;
    if (relu_x && ldrx < F) return GALA_ERR_INVALID_ARG;
    if ((relu_pro || relu_x) &&
        (A->val || (flags & GALA_SPMM_SAMPLE) || Y2 || (A->split && A->split->n_rows_split > 0)))
        return GALA_ERR_UNSUPPORTED;
    if (A->n_rows == 0 || F == 0) return GALA_OK;
    if (!Y || (!X && A->nnz > 0)) return GALA_ERR_INVALID_ARG;
    const bool samp = (flags & GALA_SPMM_SAMPLE) != 0;
    if (samp && nsamp < 0) return GALA_ERR_INVALID_ARG;
    const bool w = A->val != nullptr;
    if (w && (A->val_heads < 1 || F % A->val_heads != 0)) return GALA_ERR_INVALID_ARG;
    if (A->val_row_scale && !w) return GALA_ERR_INVALID_ARG;
    const int32_t H = w ? A->val_heads : 1, D = F / H;
    const bool accum = (flags & GALA_SPMM_ACCUM) != 0;
    const float *rs = A->val_row_scale;  // factored values: w = val * rs[row] (rounded)
#pragma omp parallel
    {
        std::vector<float> acc((size_t)F);
#pragma omp for schedule(dynamic, kRowChunk)
        for (int64_t r = 0; r < A->n_rows; ++r) {
            float *a = acc.data();
            float *yr = Y + r * ldy;
            if (accum && !dst_scale && !dst_deg)
                memcpy(a, yr, sizeof(float) * (size_t)F);
            else
                std::fill(a, a + F, 0.0f);
            for (int32_t s = 0; s < A->n_seg; ++s) {
                int64_t e0, e1;
                row_range(A, s, r, e0, e1);
                const int32_t deg = (int32_t)(e1 - e0);
                const int32_t n = samp ? (deg > 0 ? nsamp : 0) : deg;
                for (int32_t ji = 0; ji < n; ++ji) {
                    const int32_t j = samp ? (ra * ji + rb) % deg : ji;  // cuda.h:313-321
                    const int64_t e = e0 + j;
                    const int64_t c = A->col[e];
                    const float *xr = X + c * ldx;
                    const float sc = src_scale ? src_scale[c] : 1.0f;
                    if (w) {
                        for (int32_t h = 0; h < H; ++h) {
                            const float wv = rs ? A->val[e * H + h] * rs[r * H + h] : A->val[e * H + h];
                            if (src_scale)
                                for (int32_t f = h * D; f < (h + 1) * D; ++f) a[f] = fmaf(wv, sc * xr[f], a[f]);
                            else
                                for (int32_t f = h * D; f < (h + 1) * D; ++f) a[f] = fmaf(wv, xr[f], a[f]);
                        }
                    } else if (relu_pro) {  // the next layer's prologue: sc * relu(act * x)
                        const float ac = src_act ? src_act[c] : 1.0f;
                        for (int32_t f = 0; f < F; ++f) {
                            float t = xr[f];
                            if (src_act) t = ac * t;
                            t = relu_t(t);
                            if (src_scale) t = sc * t;
                            a[f] = a[f] + t;
                        }
                    } else if (src_scale) {
                        for (int32_t f = 0; f < F; ++f) a[f] = a[f] + sc * xr[f];
                    } else {
                        for (int32_t f = 0; f < F; ++f) a[f] = a[f] + xr[f];
                    }
                }
            }
            const float ds = dst_deg ? 1.0f / sqrtf((float)(A->rowptr[r + 1] - A->rowptr[r]))
                                     : (dst_scale ? dst_scale[r] : 1.0f);
            if (dst_scale || dst_deg) {
                if (accum)
                    for (int32_t f = 0; f < F; ++f) yr[f] = yr[f] + ds * a[f];
                else
                    for (int32_t f = 0; f < F; ++f) yr[f] = ds * a[f];
            } else {
                memcpy(yr, a, sizeof(float) * (size_t)F);
            }
            if (relu_x) {  // the ReLU backward of the layer's input (gala_cpu_relu_scale_backward_f32)
                const float ra_ = relu_act ? relu_act[r] : 1.0f;
                for (int32_t f = 0; f < F; ++f) {
                    float t = relu_x[r * ldrx + f];
                    if (relu_act) t = ra_ * t;
                    float d = relu_t(t) <= 0.0f ? 0.0f : yr[f];
                    if (relu_act) d = d * ra_;
                    yr[f] = d;
                }
            }
            if (Y2) {  // the next aggregation's pre-scaled input
                const float s2 = y2s ? y2s[r] : ds;
                for (int32_t f = 0; f < F; ++f) Y2[r * ldy2 + f] = s2 * yr[f];
            }
        }
    }
    return GALA_OK;
}

extern "C" int gala_cpu_degree_f32(const gala_csr_t *A, float *deg, float power, int32_t flags,
                                   int32_t nsamp, void *) {
    int st = check_csr(A);
    if (st) return st;
    if (!deg || (flags & ~(GALA_SPMM_SAMPLE))) return GALA_ERR_INVALID_ARG;
    const bool samp = (flags & GALA_SPMM_SAMPLE) != 0;
#pragma omp parallel for schedule(static, 4096)
    for (int64_t r = 0; r < A->n_rows; ++r) {
        float d;
        if (samp) {
            d = (float)nsamp * (float)A->n_seg;  // FULL_OP n * S (common.h:1358-1359)
        } else if (A->val) {
            d = 0.0f;
            for (int32_t s = 0; s < A->n_seg; ++s) {
                int64_t e0, e1;
                row_range(A, s, r, e0, e1);
                for (int64_t e = e0; e < e1; ++e) d = d + A->val[e];
            }
        } else {
            int64_t cnt = 0;
            for (int32_t s = 0; s < A->n_seg; ++s) {
                int64_t e0, e1;
                row_range(A, s, r, e0, e1);
                cnt += e1 - e0;
            }
            d = (float)cnt;
        }
        if (power != 1.0f) d = (power == -0.5f) ? 1.0f / sqrtf(d) : powf(d, power);
        deg[r] = d;
    }
    return GALA_OK;
}

extern "C" int gala_cpu_row_broadcast_f32(int64_t n_rows, int32_t F, const float *scale,
                                          const float *X, int64_t ldx, float *Y, int64_t ldy,
                                          void *) {
    if (n_rows < 0 || F < 0 || ldx < F || ldy < F) return GALA_ERR_INVALID_ARG;
    if (n_rows == 0 || F == 0) return GALA_OK;
    if (!scale || !X || !Y) return GALA_ERR_INVALID_ARG;
#pragma omp parallel for schedule(static, 1024)
    for (int64_t r = 0; r < n_rows; ++r) {
        const float s = scale[r];
        for (int32_t f = 0; f < F; ++f) Y[r * ldy + f] = s * X[r * ldx + f];
    }
    return GALA_OK;
}

extern "C" int gala_cpu_row_broadcast_deg_f32(const gala_csr_t *A, int32_t F, const float *X, int64_t ldx,
                                              float *Y, int64_t ldy, void *) {
    int st = check_csr(A);
    if (st) return st;
    if (F < 0 || ldx < F || ldy < F) return GALA_ERR_INVALID_ARG;
    if (A->n_seg != 1 || A->val) return GALA_ERR_UNSUPPORTED;  // rowptr counts: unweighted degree only
    if (A->n_rows == 0 || F == 0) return GALA_OK;
    if (!X || !Y) return GALA_ERR_INVALID_ARG;
#pragma omp parallel for schedule(static, 1024)
    for (int64_t r = 0; r < A->n_rows; ++r) {
        const float s = 1.0f / sqrtf((float)(A->rowptr[r + 1] - A->rowptr[r]));
        for (int32_t f = 0; f < F; ++f) Y[r * ldy + f] = s * X[r * ldx + f];
    }
    return GALA_OK;
}

extern "C" int gala_cpu_row_scale_relu_f32(int64_t n_rows, int32_t F, const float *act,
                                           const float *pre, const float *X, int64_t ldx,
                                           float *Y, int64_t ldy, void *) {
    if (n_rows < 0 || F < 0 || ldx < F || ldy < F) return GALA_ERR_INVALID_ARG;
    if (n_rows == 0 || F == 0) return GALA_OK;
    if (!X || !Y) return GALA_ERR_INVALID_ARG;
#pragma omp parallel for schedule(static, 1024)
    for (int64_t r = 0; r < n_rows; ++r) {
        const float a = act ? act[r] : 1.0f, b = pre ? pre[r] : 1.0f;
        for (int32_t f = 0; f < F; ++f) {
            float t = X[r * ldx + f];
            if (act) t = a * t;
            t = relu_t(t);
            if (pre) t = b * t;
            Y[r * ldy + f] = t;
        }
    }
    return GALA_OK;
}

extern "C" int gala_cpu_relu_scale_backward_f32(int64_t n_rows, int32_t F, const float *act,
                                                const float *X, int64_t ldx, const float *G,
                                                int64_t ldg, float *dX, int64_t lddx, void *) {
    if (n_rows < 0 || F < 0 || ldx < F || ldg < F || lddx < F) return GALA_ERR_INVALID_ARG;
    if (n_rows == 0 || F == 0) return GALA_OK;
    if (!X || !G || !dX) return GALA_ERR_INVALID_ARG;
#pragma omp parallel for schedule(static, 1024)
    for (int64_t r = 0; r < n_rows; ++r) {
        const float a = act ? act[r] : 1.0f;
        for (int32_t f = 0; f < F; ++f) {
            float t = X[r * ldx + f];
            if (act) t = a * t;
            float d = relu_t(t) <= 0.0f ? 0.0f : G[r * ldg + f];
            if (act) d = d * a;
            dX[r * lddx + f] = d;
        }
    }
    return GALA_OK;
}

extern "C" int gala_cpu_ffn_fwd_f32(int64_t n_rows, int32_t K, int32_t M, const float *X,
                                    int64_t ldx, const float *W, const float *b, float *Y,
                                    int64_t ldy, void *) {
    if (n_rows < 0 || K < 0 || M < 0 || ldx < K || ldy < M) return GALA_ERR_INVALID_ARG;
    if (n_rows == 0 || M == 0) return GALA_OK;
    const int wm = (M + 31) / 32;
    if (wm > 8 || (int64_t)((K + 1) & ~1) * 32 * wm > 16384) return GALA_ERR_UNSUPPORTED;
    if (!Y || (K > 0 && (!X || !W))) return GALA_ERR_INVALID_ARG;
    // bias first, then the products in k order.  The GPU kernel runs
    // v_mfma_f32_32x32x2_f32, which adds two products per step with its own internal
    // rounding, so CPU and GPU agree within fp32 summation tolerance, not bit for bit.
#pragma omp parallel for schedule(static, 256)
    for (int64_t n = 0; n < n_rows; ++n)
        for (int32_t m = 0; m < M; ++m) {
            float acc = b ? b[m] : 0.0f;
            for (int32_t k = 0; k < K; ++k) acc = fmaf(X[n * ldx + k], W[(int64_t)m * K + k], acc);
            Y[n * ldy + m] = acc;
        }
    return GALA_OK;
}

extern "C" int gala_cpu_sddvv_f32(const gala_csr_t *A, const float *a_row, const float *b_col,
                                  int32_t heads, int32_t op, float slope, float *out_e, void *) {
    int st = check_csr(A);
    if (st) return st;
    if (heads < 1) return GALA_ERR_INVALID_ARG;
    if (op < GALA_SDDVV_ADD || op > GALA_SDDVV_ADD_LRELU) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0 || A->nnz == 0) return GALA_OK;
    if (!a_row || !b_col || !out_e) return GALA_ERR_INVALID_ARG;
    const int32_t H = heads;
#pragma omp parallel for schedule(dynamic, kRowChunk)
    for (int64_t r = 0; r < A->n_rows; ++r)
        for (int32_t s = 0; s < A->n_seg; ++s) {
            int64_t e0, e1;
            row_range(A, s, r, e0, e1);
            for (int64_t e = e0; e < e1; ++e) {
                const int64_t c = A->col[e];
                for (int32_t h = 0; h < H; ++h) {
                    const float av = a_row[r * H + h], bv = b_col[c * H + h];
                    float v;
                    if (op == GALA_SDDVV_MUL) {
                        v = av * bv;
                    } else {
                        v = av + bv;
                        if (op == GALA_SDDVV_ADD_LRELU) v = v > 0.0f ? v : v * slope;
                    }
                    out_e[e * H + h] = v;
                }
            }
        }
    return GALA_OK;
}

extern "C" int gala_cpu_row_sum_f32(const gala_csr_t *A, const float *v_e, int32_t heads,
                                    float eps, float *out_row, int32_t flags, void *) {
    int st = check_csr(A);
    if (st) return st;
    // GALA_SPMM_HUB_CHUNKED is accepted (the HIP library's fast mode); every row here is
    // one sequential pass, the reference's order
    if (heads < 1 || (flags & ~(GALA_SPMM_ACCUM | GALA_SPMM_HUB_CHUNKED))) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0) return GALA_OK;
    if (!out_row || (!v_e && A->nnz > 0)) return GALA_ERR_INVALID_ARG;
    const bool accum = (flags & GALA_SPMM_ACCUM) != 0;
    const int32_t H = heads;
#pragma omp parallel for schedule(dynamic, kRowChunk)
    for (int64_t r = 0; r < A->n_rows; ++r)
        for (int32_t h = 0; h < H; ++h) {
            float c = accum ? out_row[r * H + h] : 0.0f;
            for (int32_t s = 0; s < A->n_seg; ++s) {
                int64_t e0, e1;
                row_range(A, s, r, e0, e1);
                float local = eps;  // each segment launch starts at 1e-12 (cuda.h:512,666)
                for (int64_t e = e0; e < e1; ++e) local = local + v_e[e * H + h];
                c = c + local;
            }
            out_row[r * H + h] = c;
        }
    return GALA_OK;
}

extern "C" int gala_cpu_row_scale_f32(const gala_csr_t *A, const float *q_row, int32_t heads,
                                      float *v_inout, void *) {
    int st = check_csr(A);
    if (st) return st;
    if (heads < 1) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0 || A->nnz == 0) return GALA_OK;
    if (!q_row || !v_inout) return GALA_ERR_INVALID_ARG;
    const int32_t H = heads;
#pragma omp parallel for schedule(dynamic, kRowChunk)
    for (int64_t r = 0; r < A->n_rows; ++r)
        for (int32_t s = 0; s < A->n_seg; ++s) {
            int64_t e0, e1;
            row_range(A, s, r, e0, e1);
            for (int64_t e = e0; e < e1; ++e)
                for (int32_t h = 0; h < H; ++h) v_inout[e * H + h] = v_inout[e * H + h] * q_row[r * H + h];
        }
    return GALA_OK;
}

extern "C" int gala_cpu_sddmm_dot_f32(const gala_csr_t *A, const float *Ad, int64_t lda,
                                      const float *Bd, int64_t ldb, int32_t F, int32_t heads,
                                      float *out_e, void *) {
    int st = check_csr(A);
    if (st) return st;
    if (heads < 1) return GALA_ERR_INVALID_ARG;
    if (F < 1 || F % heads != 0 || lda < F || ldb < F) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0 || A->nnz == 0) return GALA_OK;
    if (!Ad || !Bd || !out_e) return GALA_ERR_INVALID_ARG;
    const int32_t H = heads, D = F / H;
#pragma omp parallel for schedule(dynamic, kRowChunk)
    for (int64_t r = 0; r < A->n_rows; ++r)
        for (int32_t s = 0; s < A->n_seg; ++s) {
            int64_t e0, e1;
            row_range(A, s, r, e0, e1);
            for (int64_t e = e0; e < e1; ++e) {
                const float *br = Bd + (int64_t)A->col[e] * ldb;
                for (int32_t h = 0; h < H; ++h) {
                    float local = 0.0f;  // cuda.h:720-727, fma contracted
                    for (int32_t k = h * D; k < (h + 1) * D; ++k) local = fmaf(Ad[r * lda + k], br[k], local);
                    out_e[e * H + h] = local;
                }
            }
        }
    return GALA_OK;
}

extern "C" int gala_cpu_edge_softmax_fwd_f32(const gala_csr_t *A, const float *logits,
                                             int32_t heads, int32_t mode, float *alpha, void *) {
    int st = check_csr(A);
    if (st) return st;
    if (heads < 1) return GALA_ERR_INVALID_ARG;
    if (mode != GALA_SOFTMAX_REF && mode != GALA_SOFTMAX_FIXED) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0 || A->nnz == 0) return GALA_OK;
    if (!logits || !alpha) return GALA_ERR_INVALID_ARG;
    const int32_t H = heads, S = A->n_seg;
#pragma omp parallel for schedule(dynamic, kRowChunk)
    for (int64_t r = 0; r < A->n_rows; ++r)
        for (int32_t h = 0; h < H; ++h) {
            float m = 0.0f, q;
            if (mode == GALA_SOFTMAX_REF) {
                // val_exp = clamp(exp(s)); row_sum = K7 (1e-12 per segment); reciprocal
                float c = 0.0f;
                for (int32_t s = 0; s < S; ++s) {
                    int64_t e0, e1;
                    row_range(A, s, r, e0, e1);
                    float local = 1e-12f;
                    for (int64_t e = e0; e < e1; ++e) local = local + ref_exp(logits[e * H + h]);
                    c = c + local;
                }
                q = 1.0f / c;
            } else {
                m = -INFINITY;
                for (int32_t s = 0; s < S; ++s) {
                    int64_t e0, e1;
                    row_range(A, s, r, e0, e1);
                    for (int64_t e = e0; e < e1; ++e) m = fmaxf(m, logits[e * H + h]);
                }
                float sum = 0.0f;
                for (int32_t s = 0; s < S; ++s) {
                    int64_t e0, e1;
                    row_range(A, s, r, e0, e1);
                    for (int64_t e = e0; e < e1; ++e) sum = sum + expf(logits[e * H + h] - m);
                }
                q = 1.0f / sum;
            }
            for (int32_t s = 0; s < S; ++s) {
                int64_t e0, e1;
                row_range(A, s, r, e0, e1);
                for (int64_t e = e0; e < e1; ++e) {
                    const float x = logits[e * H + h];
                    const float pe = mode == GALA_SOFTMAX_REF ? ref_exp(x) : expf(x - m);
                    alpha[e * H + h] = pe * q;
                }
            }
        }
    return GALA_OK;
}

extern "C" int gala_cpu_edge_softmax_bwd_f32(const gala_csr_t *A, const float *alpha,
                                             const float *d_alpha, int32_t heads, int32_t mode,
                                             float *d_logits, void *) {
    int st = check_csr(A);
    if (st) return st;
    if (heads < 1) return GALA_ERR_INVALID_ARG;
    if (mode != GALA_SOFTMAX_REF && mode != GALA_SOFTMAX_FIXED) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0 || A->nnz == 0) return GALA_OK;
    if (!alpha || !d_alpha || !d_logits) return GALA_ERR_INVALID_ARG;
    const int32_t H = heads, S = A->n_seg;
    const float eps = mode == GALA_SOFTMAX_REF ? 1e-12f : 0.0f;
#pragma omp parallel for schedule(dynamic, kRowChunk)
    for (int64_t r = 0; r < A->n_rows; ++r)
        for (int32_t h = 0; h < H; ++h) {
            float c = 0.0f;  // accum = K7(sds) (common.h:793-794)
            for (int32_t s = 0; s < S; ++s) {
                int64_t e0, e1;
                row_range(A, s, r, e0, e1);
                float local = eps;
                for (int64_t e = e0; e < e1; ++e) local = local + alpha[e * H + h] * d_alpha[e * H + h];
                c = c + local;
            }
            for (int32_t s = 0; s < S; ++s) {
                int64_t e0, e1;
                row_range(A, s, r, e0, e1);
                for (int64_t e = e0; e < e1; ++e) {
                    const float a = alpha[e * H + h];
                    d_logits[e * H + h] = a * d_alpha[e * H + h] - a * c;  // sds - K8(accum)
                }
            }
        }
    return GALA_OK;
}

static int cpu_gat_fwd(const gala_csr_t *A, const float *aL, const float *aR, const float *X,
                       int64_t ldx, int32_t F, int32_t heads, float slope, int32_t mode, float *Y,
                       int64_t ldy, float *alpha_out, float *q_out) {
    const bool partial = (mode & GALA_GAT_PARTIAL) != 0;  // see gala_hip.h
    mode &= ~GALA_GAT_PARTIAL;
    if (partial && (mode != GALA_SOFTMAX_REF || !q_out || alpha_out)) return GALA_ERR_INVALID_ARG;
    int st = check_csr(A);
    if (st) return st;
    if (heads < 1) return GALA_ERR_INVALID_ARG;
    if (mode != GALA_SOFTMAX_REF && mode != GALA_SOFTMAX_FIXED) return GALA_ERR_INVALID_ARG;
    if (F < 1 || F % heads != 0 || ldx < F || ldy < F) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0) return GALA_OK;
    if (!aL || !aR || !Y || (!X && A->nnz > 0)) return GALA_ERR_INVALID_ARG;
    const int32_t H = heads, D = F / H, S = A->n_seg;
#pragma omp parallel
    {
        std::vector<float> acc((size_t)D);
#pragma omp for schedule(dynamic, kRowChunk)
        for (int64_t r = 0; r < A->n_rows; ++r)
            for (int32_t h = 0; h < H; ++h) {
                const float al = aL[r * H + h];
                auto logit = [&](int64_t e) {
                    float z = al + aR[(int64_t)A->col[e] * H + h];
                    return z > 0.0f ? z : z * slope;  // LeakyReLU (common.h:1175-1184)
                };
                float m = 0.0f;
                if (mode == GALA_SOFTMAX_FIXED) {
                    m = -INFINITY;
                    for (int32_t s = 0; s < S; ++s) {
                        int64_t e0, e1;
                        row_range(A, s, r, e0, e1);
                        for (int64_t e = e0; e < e1; ++e) m = fmaxf(m, logit(e));
                    }
                }
                std::fill(acc.begin(), acc.end(), 0.0f);
                float sum = 0.0f;
                for (int32_t s = 0; s < S; ++s) {
                    int64_t e0, e1;
                    row_range(A, s, r, e0, e1);
                    for (int64_t e = e0; e < e1; ++e) {
                        const float z = logit(e);
                        const float pe = mode == GALA_SOFTMAX_REF ? ref_exp(z) : expf(z - m);
                        sum = sum + pe;
                        const float *xr = X + (int64_t)A->col[e] * ldx + h * D;
                        for (int32_t f = 0; f < D; ++f) acc[f] = fmaf(pe, xr[f], acc[f]);
                    }
                }
                const float den = mode == GALA_SOFTMAX_REF ? sum + (float)S * 1e-12f : sum;
                const float q = 1.0f / den;
                const bool empty = mode != GALA_SOFTMAX_REF && sum == 0.0f;
                for (int32_t f = 0; f < D; ++f) Y[r * ldy + h * D + f] = partial ? acc[f] : empty ? 0.0f : acc[f] * q;
                if (q_out) q_out[r * H + h] = partial ? sum : q;
                if (!alpha_out) continue;
                for (int32_t s = 0; s < S; ++s) {
                    int64_t e0, e1;
                    row_range(A, s, r, e0, e1);
                    for (int64_t e = e0; e < e1; ++e) {
                        const float z = logit(e);
                        const float pe = mode == GALA_SOFTMAX_REF ? ref_exp(z) : expf(z - m);
                        alpha_out[e * H + h] = q_out ? pe : pe * q;
                    }
                }
            }
    }
    return GALA_OK;
}

extern "C" int gala_cpu_gat_fwd_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                    const float *X, int64_t ldx, int32_t F, int32_t heads,
                                    float slope, int32_t mode, float *Y, int64_t ldy,
                                    float *alpha_out, void *) {
    return cpu_gat_fwd(A, aL, aR, X, ldx, F, heads, slope, mode, Y, ldy, alpha_out, nullptr);
}

static int cpu_gat_bwd(const gala_csr_t *A, const float *aL, const float *aR, const float *X,
                       int64_t ldx, const float *dY, int64_t lddy, int32_t F, int32_t heads,
                       float slope, int32_t mode, const float *alpha, const float *q,
                       float *d_logit, float *d_aL) {
    int st = check_csr(A);
    if (st) return st;
    if (heads < 1) return GALA_ERR_INVALID_ARG;
    if (mode != GALA_SOFTMAX_REF && mode != GALA_SOFTMAX_FIXED) return GALA_ERR_INVALID_ARG;
    if (F < 1 || F % heads != 0 || ldx < F || lddy < F) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0) return GALA_OK;
    if (!aL || !aR || !dY || !d_aL || (A->nnz > 0 && (!X || !alpha))) return GALA_ERR_INVALID_ARG;
    if (mode == GALA_SOFTMAX_FIXED && !d_logit && A->nnz > 0) return GALA_ERR_INVALID_ARG;
    const int32_t H = heads, D = F / H, S = A->n_seg;
    const float eps = mode == GALA_SOFTMAX_REF ? 1e-12f : 0.0f;
#pragma omp parallel
    {
        std::vector<float> sds;
#pragma omp for schedule(dynamic, kRowChunk)
        for (int64_t r = 0; r < A->n_rows; ++r)
            for (int32_t h = 0; h < H; ++h) {
                const float *dyr = dY + r * lddy + h * D;
                const float qrh = q ? q[r * H + h] : 1.0f;
                // factored attention (p, q): alpha = p * q, rounded like the materialised one
                auto alp = [&](int64_t e) { return q ? alpha[e * H + h] * qrh : alpha[e * H + h]; };
                // d alpha = edge_sddmm (cuda.h:808-845); sds = alpha*d alpha; acc = K7(sds)
                float c = 0.0f;
                sds.clear();
                for (int32_t s = 0; s < S; ++s) {
                    int64_t e0, e1;
                    row_range(A, s, r, e0, e1);
                    float local = eps;
                    for (int64_t e = e0; e < e1; ++e) {
                        const float *xr = X + (int64_t)A->col[e] * ldx + h * D;
                        float d = 0.0f;
                        for (int32_t k = 0; k < D; ++k) d = fmaf(dyr[k], xr[k], d);
                        const float v = alp(e) * d;
                        sds.push_back(v);
                        local = local + v;
                    }
                    c = c + local;
                }
                // ds = sds - alpha*acc; LeakyReLU backward; K7 row sum of dz
                float c2 = 0.0f;
                size_t i = 0;
                for (int32_t s = 0; s < S; ++s) {
                    int64_t e0, e1;
                    row_range(A, s, r, e0, e1);
                    float local = eps;
                    for (int64_t e = e0; e < e1; ++e, ++i) {
                        const float ds = sds[i] - alp(e) * c;
                        const float z = aL[r * H + h] + aR[(int64_t)A->col[e] * H + h];
                        const float dz = z > 0.0f ? ds : ds * slope;
                        if (d_logit) d_logit[e * H + h] = dz;
                        local = local + dz;
                    }
                    c2 = c2 + local;
                }
                d_aL[r * H + h] = c2;
            }
    }
    return GALA_OK;
}

extern "C" int gala_cpu_gat_bwd_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                    const float *X, int64_t ldx, const float *dY, int64_t lddy,
                                    int32_t F, int32_t heads, float slope, int32_t mode,
                                    const float *alpha, float *d_logit, float *d_aL, void *) {
    return cpu_gat_bwd(A, aL, aR, X, ldx, dY, lddy, F, heads, slope, mode, alpha, nullptr, d_logit,
                       d_aL);
}

// aR[j] = <X[j, 0:F], wR> + bR: the attention Linear the *_attn entry points recompute
static std::vector<float> attn_logits(const gala_csr_t *A, const float *wR, const float *bR,
                                      const float *X, int64_t ldx, int32_t F) {
    std::vector<float> aR((size_t)A->n_cols);
    const float b = bR ? bR[0] : 0.0f;
#pragma omp parallel for schedule(static, 4096)
    for (int64_t j = 0; j < A->n_cols; ++j) {
        float d = 0.0f;
        for (int32_t f = 0; f < F; ++f) d = fmaf(wR[f], X[j * ldx + f], d);
        aR[(size_t)j] = d + b;
    }
    return aR;
}

extern "C" int gala_cpu_gat_fwd_attn_f32(const gala_csr_t *A, const float *aL, const float *wR,
                                         const float *bR, const float *X, int64_t ldx, int32_t F,
                                         float slope, int32_t mode, float *Y, int64_t ldy,
                                         float *alpha_out, void *stream) {
    int st = check_csr(A);
    if (st) return st;
    if (F < 1 || ldx < F) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0) return GALA_OK;
    if (!wR || (!X && A->n_cols > 0)) return GALA_ERR_INVALID_ARG;
    const std::vector<float> aR = attn_logits(A, wR, bR, X, ldx, F);
    return gala_cpu_gat_fwd_f32(A, aL, aR.data(), X, ldx, F, 1, slope, mode, Y, ldy, alpha_out,
                                stream);
}

extern "C" int gala_cpu_gat_bwd_attn_f32(const gala_csr_t *A, const float *aL, const float *wR,
                                         const float *bR, const float *X, int64_t ldx,
                                         const float *dY, int64_t lddy, int32_t F, float slope,
                                         const float *alpha, float *d_aL, void *stream) {
    int st = check_csr(A);
    if (st) return st;
    if (F < 1 || ldx < F) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0) return GALA_OK;
    if (!wR || (!X && A->n_cols > 0)) return GALA_ERR_INVALID_ARG;
    const std::vector<float> aR = attn_logits(A, wR, bR, X, ldx, F);
    return gala_cpu_gat_bwd_f32(A, aL, aR.data(), X, ldx, dY, lddy, F, 1, slope, GALA_SOFTMAX_REF,
                                alpha, nullptr, d_aL, stream);
}

// aR[j,h] = <X[j, hD:(h+1)D], wR[hD:(h+1)D]> + bR[h]: the per-head attention logits of
// the ex entry points' recompute (one head: attn_logits)
static std::vector<float> attn_logits_heads(const gala_csr_t *A, const float *wR, const float *bR,
                                            const float *X, int64_t ldx, int32_t F, int32_t H) {
    std::vector<float> aR((size_t)A->n_cols * H);
    const int32_t D = F / H;
#pragma omp parallel for schedule(static, 4096)
    for (int64_t j = 0; j < A->n_cols; ++j)
        for (int32_t h = 0; h < H; ++h) {
            float d = 0.0f;
            for (int32_t f = h * D; f < (h + 1) * D; ++f) d = fmaf(wR[f], X[j * ldx + f], d);
            aR[(size_t)j * H + h] = d + (bR ? bR[h] : 0.0f);
        }
    return aR;
}

extern "C" int gala_cpu_gat_fwd_ex_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                       const float *wR, const float *bR, const float *X,
                                       int64_t ldx, int32_t F, int32_t heads, float slope,
                                       int32_t mode, float *Y, int64_t ldy, float *alpha_out,
                                       float *q_out, void *) {
    int st = check_csr(A);
    if (st) return st;
    if (heads < 1 || F < 1 || F % heads != 0 || ldx < F) return GALA_ERR_INVALID_ARG;
    if (q_out && (mode & ~GALA_GAT_PARTIAL) != GALA_SOFTMAX_REF) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0) return GALA_OK;
    if (!aR && (!wR || (!X && A->n_cols > 0))) return GALA_ERR_INVALID_ARG;
    std::vector<float> rc;
    if (!aR) {
        rc = attn_logits_heads(A, wR, bR, X, ldx, F, heads);
        aR = rc.data();
    }
    return cpu_gat_fwd(A, aL, aR, X, ldx, F, heads, slope, mode, Y, ldy, alpha_out, q_out);
}

extern "C" int gala_cpu_gat_bwd_ex_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                       const float *wR, const float *bR, const float *X,
                                       int64_t ldx, const float *dY, int64_t lddy, int32_t F,
                                       int32_t heads, float slope, int32_t mode, const float *alpha,
                                       const float *q, float *d_logit, float *d_aL, void *) {
    int st = check_csr(A);
    if (st) return st;
    if (heads < 1 || F < 1 || F % heads != 0 || ldx < F) return GALA_ERR_INVALID_ARG;
    if (q && mode != GALA_SOFTMAX_REF) return GALA_ERR_INVALID_ARG;
    if (!aR && mode != GALA_SOFTMAX_REF) return GALA_ERR_UNSUPPORTED;
    if (A->n_rows == 0) return GALA_OK;
    if (!aR && (!wR || (!X && A->n_cols > 0))) return GALA_ERR_INVALID_ARG;
    std::vector<float> rc;
    if (!aR) {
        rc = attn_logits_heads(A, wR, bR, X, ldx, F, heads);
        aR = rc.data();
    }
    return cpu_gat_bwd(A, aL, aR, X, ldx, dY, lddy, F, heads, slope, mode, alpha, q, d_logit, d_aL);
}

extern "C" int gala_cpu_gat_bwd_fused_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                          const float *wR, const float *bR, const float *X,
                                          int64_t ldx, const float *dY, int64_t lddy, int32_t F,
                                          int32_t heads, float slope, const float *q, float *dX,
                                          int64_t lddx, float *d_aL, void *) {
    int st = check_csr(A);
    if (st) return st;
    if (heads < 1 || F < 1 || F % heads != 0 || ldx < F || lddy < F || lddx < F) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0) return GALA_OK;
    if (!aL || (!aR && !wR) || !q || !dY || !dX || !d_aL || (A->nnz > 0 && !X)) return GALA_ERR_INVALID_ARG;
    if (A->n_cols > A->n_rows && A->nnz > 0) return GALA_ERR_INVALID_ARG;
    std::vector<float> rc;
    if (!aR) {
        rc = attn_logits_heads(A, wR, bR, X, ldx, F, heads);
        aR = rc.data();
    }
    const int32_t H = heads, D = F / H, S = A->n_seg;
    // the recomputed alpha = fl(p * q), materialised on the host
    std::vector<float> alpha((size_t)A->nnz * H);
#pragma omp parallel for schedule(dynamic, kRowChunk)
    for (int64_t r = 0; r < A->n_rows; ++r)
        for (int32_t s = 0; s < S; ++s) {
            int64_t e0, e1;
            row_range(A, s, r, e0, e1);
            for (int64_t e = e0; e < e1; ++e)
                for (int32_t h = 0; h < H; ++h) {
                    float z = aL[r * H + h] + aR[(int64_t)A->col[e] * H + h];
                    z = z > 0.0f ? z : z * slope;
                    alpha[(size_t)e * H + h] = ref_exp(z) * q[r * H + h];
                }
        }
    // dX = A_alpha dY on the forward pattern (sequential fma per row, the SpMM's order)
#pragma omp parallel for schedule(dynamic, kRowChunk)
    for (int64_t r = 0; r < A->n_rows; ++r) {
        float *out = dX + r * lddx;
        for (int32_t f = 0; f < F; ++f) out[f] = 0.0f;
        for (int32_t s = 0; s < S; ++s) {
            int64_t e0, e1;
            row_range(A, s, r, e0, e1);
            for (int64_t e = e0; e < e1; ++e) {
                const float *yr = dY + (int64_t)A->col[e] * lddy;
                for (int32_t h = 0; h < H; ++h) {
                    const float w = alpha[(size_t)e * H + h];
                    for (int32_t f = h * D; f < (h + 1) * D; ++f) out[f] = fmaf(w, yr[f], out[f]);
                }
            }
        }
    }
    return cpu_gat_bwd(A, aL, aR, X, ldx, dY, lddy, F, heads, slope, GALA_SOFTMAX_REF, alpha.data(), nullptr,
                       nullptr, d_aL);
}

// REF forward with the row statistics (gala_hip.h, gala_gat_fwd_stats_f32): Y and q as
// cpu_gat_fwd, plus Ym = q * sum m p X and sma = q * sum m p (m the LeakyReLU factor)
// partial (vertex cut): every output unnormalised (Y = sum p X, q_out = sum p, Ym = sum m p X,
// sma = sum m p), for the rows' owners to add first (gala_cpu_gat_fwd_partial_stats_f32)
static int cpu_gat_fwd_stats(const gala_csr_t *A, const float *aL, const float *aR, const float *wR,
                             const float *bR, const float *X, int64_t ldx, int32_t F, int32_t heads,
                             float slope, float *Y, int64_t ldy, float *q_out, float *Ym, int64_t ldym,
                             float *sma, float *aR_out, float *p_out, bool partial,
                             const int32_t *self_col = nullptr) {
    int st = check_csr(A);
    if (st) return st;
    if (heads < 1 || F < 1 || F % heads != 0 || ldx < F || ldy < F || ldym < F) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0) return GALA_OK;
    if (!aL || (!aR && !wR) || !Y || !q_out || !Ym || !sma || (!X && A->nnz > 0)) return GALA_ERR_INVALID_ARG;
    if (!partial && !self_col && A->n_cols > A->n_rows && A->nnz > 0) return GALA_ERR_INVALID_ARG;
    if (aR_out && (aR || !X || (partial && !self_col))) return GALA_ERR_INVALID_ARG;
    std::vector<float> rc;
    if (!aR) {
        rc = attn_logits_heads(A, wR, bR, X, ldx, F, heads);
        aR = rc.data();
        if (aR_out && !self_col) std::copy(rc.begin(), rc.begin() + A->n_rows * heads, aR_out);
        if (aR_out && self_col)  // the own vertices' logits (a vertex cut's rows are not its columns)
            for (int64_t r = 0; r < A->n_rows; ++r)
                if (self_col[r] >= 0)
                    std::copy(rc.begin() + (int64_t)self_col[r] * heads, rc.begin() + ((int64_t)self_col[r] + 1) * heads,
                              aR_out + (int64_t)self_col[r] * heads);
    }
    const int32_t H = heads, D = F / H, S = A->n_seg;
#pragma omp parallel
    {
        std::vector<float> acc((size_t)D), accm((size_t)D);
#pragma omp for schedule(dynamic, kRowChunk)
        for (int64_t r = 0; r < A->n_rows; ++r)
            for (int32_t h = 0; h < H; ++h) {
                std::fill(acc.begin(), acc.end(), 0.0f);
                std::fill(accm.begin(), accm.end(), 0.0f);
                float sum = 0.0f, sm = 0.0f;
                for (int32_t s = 0; s < S; ++s) {
                    int64_t e0, e1;
                    row_range(A, s, r, e0, e1);
                    for (int64_t e = e0; e < e1; ++e) {
                        const float t = aL[r * H + h] + aR[(int64_t)A->col[e] * H + h];
                        const bool pos = t > 0.0f;
                        const float pe = ref_exp(pos ? t : t * slope);
                        const float mp = pos ? pe : pe * slope;
                        if (p_out) p_out[e * H + h] = pe;
                        sum = sum + pe;
                        sm = sm + mp;
                        const float *xr = X + (int64_t)A->col[e] * ldx + h * D;
                        for (int32_t f = 0; f < D; ++f) {
                            acc[f] = fmaf(pe, xr[f], acc[f]);
                            accm[f] = fmaf(mp, xr[f], accm[f]);
                        }
                    }
                }
                const float q = partial ? 1.0f : 1.0f / (sum + (float)S * 1e-12f);
                for (int32_t f = 0; f < D; ++f) {
                    Y[r * ldy + h * D + f] = partial ? acc[f] : acc[f] * q;
                    Ym[r * ldym + h * D + f] = partial ? accm[f] : accm[f] * q;
                }
                q_out[r * H + h] = partial ? sum : q;
                sma[r * H + h] = partial ? sm : sm * q;
            }
    }
    return GALA_OK;
}

extern "C" int gala_cpu_gat_fwd_stats_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                          const float *wR, const float *bR, const float *X,
                                          int64_t ldx, int32_t F, int32_t heads, float slope, float *Y,
                                          int64_t ldy, float *q_out, float *Ym, int64_t ldym, float *sma,
                                          float *aR_out, float *p_out, void *) {
    return cpu_gat_fwd_stats(A, aL, aR, wR, bR, X, ldx, F, heads, slope, Y, ldy, q_out, Ym, ldym, sma, aR_out,
                             p_out, false);
}

extern "C" int gala_cpu_gat_fwd_partial_stats_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                                  const float *wR, const float *bR, const float *X,
                                                  int64_t ldx, int32_t F, int32_t heads, float slope, float *U,
                                                  int64_t ldu, float *sums, float *Um, int64_t ldum,
                                                  float *msums, void *) {
    return cpu_gat_fwd_stats(A, aL, aR, wR, bR, X, ldx, F, heads, slope, U, ldu, sums, Um, ldum, msums, nullptr,
                             nullptr, true);
}

extern "C" int gala_cpu_gat_fwd_partial_stats_ex_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                                     const float *wR, const float *bR, const float *X,
                                                     int64_t ldx, int32_t F, int32_t heads, float slope, float *U,
                                                     int64_t ldu, float *sums, float *Um, int64_t ldum,
                                                     float *msums, const int32_t *self_col, float *aR_out, void *) {
    if (aR_out && !self_col) return GALA_ERR_INVALID_ARG;
    return cpu_gat_fwd_stats(A, aL, aR, wR, bR, X, ldx, F, heads, slope, U, ldu, sums, Um, ldum, msums, aR_out,
                             nullptr, true, self_col);
}

// gala_gat_fwd_continue_f32 (gala_hip.h): every row's sums start at the partials of an
// earlier pass over other columns (which may alias the outputs), then take this pattern's
// edges in CSR order; Ym NULL: the plain REF forward; flags GALA_GAT_PARTIAL: unnormalised
extern "C" int gala_cpu_gat_fwd_continue_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                             const float *wR, const float *bR, const float *X, int64_t ldx,
                                             int32_t F, int32_t heads, float slope, int32_t flags,
                                             const float *U0, int64_t ldu0, const float *S0, const float *Um0, int64_t ldum0,
                                             const float *M0, float *Y, int64_t ldy, float *q_out, float *Ym,
                                             int64_t ldym, float *sma, void *) {
    int st = check_csr(A);
    if (st) return st;
    const bool stats = Ym != nullptr, partial = flags == GALA_GAT_PARTIAL;
    if (flags != 0 && !partial) return GALA_ERR_INVALID_ARG;
    if (heads < 1 || F < 1 || F % heads != 0 || ldx < F || ldy < F || ldu0 < F) return GALA_ERR_INVALID_ARG;
    if ((Um0 != nullptr) != stats || (stats && (ldym < F || ldum0 < F || !M0 || !sma || !q_out)))
        return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0) return GALA_OK;
    if (!aL || (!aR && !wR) || !Y || !U0 || !S0 || (!X && A->nnz > 0)) return GALA_ERR_INVALID_ARG;
    std::vector<float> rc;
    if (!aR) {
        rc = attn_logits_heads(A, wR, bR, X, ldx, F, heads);
        aR = rc.data();
    }
    const int32_t H = heads, D = F / H, S = A->n_seg;
#pragma omp parallel
    {
        std::vector<float> acc((size_t)D), accm((size_t)D);
#pragma omp for schedule(dynamic, kRowChunk)
        for (int64_t r = 0; r < A->n_rows; ++r)
            for (int32_t h = 0; h < H; ++h) {
                std::copy(U0 + r * ldu0 + h * D, U0 + r * ldu0 + (h + 1) * D, acc.begin());
                if (stats) std::copy(Um0 + r * ldum0 + h * D, Um0 + r * ldum0 + (h + 1) * D, accm.begin());
                float sum = S0[r * H + h], sm = stats ? M0[r * H + h] : 0.0f;
                for (int32_t s = 0; s < S; ++s) {
                    int64_t e0, e1;
                    row_range(A, s, r, e0, e1);
                    for (int64_t e = e0; e < e1; ++e) {
                        const float t = aL[r * H + h] + aR[(int64_t)A->col[e] * H + h];
                        const bool pos = t > 0.0f;
                        const float pe = ref_exp(pos ? t : t * slope);
                        const float mp = pos ? pe : pe * slope;
                        sum = sum + pe;
                        sm = sm + mp;
                        const float *xr = X + (int64_t)A->col[e] * ldx + h * D;
                        for (int32_t f = 0; f < D; ++f) {
                            acc[f] = fmaf(pe, xr[f], acc[f]);
                            if (stats) accm[f] = fmaf(mp, xr[f], accm[f]);
                        }
                    }
                }
                const float q = partial ? 1.0f : 1.0f / (sum + (float)S * 1e-12f);
                for (int32_t f = 0; f < D; ++f) Y[r * ldy + h * D + f] = partial ? acc[f] : acc[f] * q;
                if (stats)
                    for (int32_t f = 0; f < D; ++f) Ym[r * ldym + h * D + f] = partial ? accm[f] : accm[f] * q;
                if (q_out) q_out[r * H + h] = partial ? sum : q;
                if (stats) sma[r * H + h] = partial ? sm : sm * q;
            }
    }
    return GALA_OK;
}

extern "C" int gala_cpu_gat_fwd_stats_ex_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                             const float *wR, const float *bR, const float *X, int64_t ldx,
                                             int32_t F, int32_t heads, float slope, float *Y, int64_t ldy,
                                             float *q_out, float *Ym, int64_t ldym, float *sma,
                                             const int32_t *self_col, float *aR_out, float *p_out, void *) {
    return cpu_gat_fwd_stats(A, aL, aR, wR, bR, X, ldx, F, heads, slope, Y, ldy, q_out, Ym, ldym, sma, aR_out,
                             p_out, false, self_col);
}

// REF backward from the row statistics: dX as gala_cpu_gat_bwd_fused_f32, d_aL from
// <dY, Y> and <dY, Ym>; dY_rows: the rows' own dY when dY is a gathered table
static int cpu_gat_bwd_stats(const gala_csr_t *A, const float *aL, const float *aR, const float *pe,
                             const float *dY, int64_t lddy, const float *dY_rows, int32_t F, int32_t heads,
                             float slope, const float *q, const float *Y, int64_t ldy, const float *Ym,
                             int64_t ldym, const float *sma, float *dX, int64_t lddx, float *d_aL) {
    int st = check_csr(A);
    if (st) return st;
    if (heads < 1 || F < 1 || F % heads != 0 || lddy < F || ldy < F || ldym < F || lddx < F)
        return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0) return GALA_OK;
    if (!aL || (!aR && !pe) || !q || !dY || !Y || !Ym || !sma || !dX || !d_aL) return GALA_ERR_INVALID_ARG;
    if (!dY_rows && A->n_cols > A->n_rows && A->nnz > 0) return GALA_ERR_INVALID_ARG;
    const float *dYr = dY_rows ? dY_rows : dY;
    const int32_t H = heads, D = F / H, S = A->n_seg;
    const float eps = (float)S * 1e-12f;
#pragma omp parallel for schedule(dynamic, kRowChunk)
    for (int64_t r = 0; r < A->n_rows; ++r) {
        float *out = dX + r * lddx;
        for (int32_t f = 0; f < F; ++f) out[f] = 0.0f;
        for (int32_t s = 0; s < S; ++s) {
            int64_t e0, e1;
            row_range(A, s, r, e0, e1);
            for (int64_t e = e0; e < e1; ++e) {
                const float *yr = dY + (int64_t)A->col[e] * lddy;
                for (int32_t h = 0; h < H; ++h) {
                    float w;
                    if (pe) {
                        w = pe[e * H + h] * q[r * H + h];
                    } else {
                        float z = aL[r * H + h] + aR[(int64_t)A->col[e] * H + h];
                        z = z > 0.0f ? z : z * slope;
                        w = ref_exp(z) * q[r * H + h];
                    }
                    for (int32_t f = h * D; f < (h + 1) * D; ++f) out[f] = fmaf(w, yr[f], out[f]);
                }
            }
        }
        for (int32_t h = 0; h < H; ++h) {
            float syy = 0.0f, sym = 0.0f;
            for (int32_t f = h * D; f < (h + 1) * D; ++f) {
                syy = fmaf(dYr[r * lddy + f], Y[r * ldy + f], syy);
                sym = fmaf(dYr[r * lddy + f], Ym[r * ldym + f], sym);
            }
            const float acc = syy + eps;
            d_aL[r * H + h] = (sym - acc * sma[r * H + h]) + eps;
        }
    }
    return GALA_OK;
}

extern "C" int gala_cpu_gat_bwd_stats_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                          const float *pe, const float *dY, int64_t lddy, int32_t F, int32_t heads,
                                          float slope, const float *q, const float *Y, int64_t ldy,
                                          const float *Ym, int64_t ldym, const float *sma, float *dX,
                                          int64_t lddx, float *d_aL, void *) {
    return cpu_gat_bwd_stats(A, aL, aR, pe, dY, lddy, nullptr, F, heads, slope, q, Y, ldy, Ym, ldym, sma, dX, lddx,
                             d_aL);
}

extern "C" int gala_cpu_gat_bwd_stats_ex_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                             const float *pe, const float *dY, int64_t lddy, const float *dY_rows,
                                             int32_t F, int32_t heads, float slope, const float *q, const float *Y,
                                             int64_t ldy, const float *Ym, int64_t ldym, const float *sma,
                                             float *dX, int64_t lddx, float *d_aL, void *) {
    return cpu_gat_bwd_stats(A, aL, aR, pe, dY, lddy, dY_rows, F, heads, slope, q, Y, ldy, Ym, ldym, sma, dX, lddx,
                             d_aL);
}

// gala_gat_bwd_stats_linear_f32 (gala_hip.h): then dX[r, f] += d_aL[r, head(f)] * wR[f]
extern "C" int gala_cpu_gat_bwd_stats_linear_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                                 const float *pe, const float *dY, int64_t lddy,
                                                 const float *dY_rows, int32_t F, int32_t heads, float slope,
                                                 const float *q, const float *Y, int64_t ldy, const float *Ym,
                                                 int64_t ldym, const float *sma, const float *wR, float *dX,
                                                 int64_t lddx, float *d_aL, void *) {
    if (!wR && A && A->n_rows > 0) return GALA_ERR_INVALID_ARG;
    const int st = cpu_gat_bwd_stats(A, aL, aR, pe, dY, lddy, dY_rows, F, heads, slope, q, Y, ldy, Ym, ldym, sma,
                                     dX, lddx, d_aL);
    if (st || A->n_rows == 0) return st;
    const int32_t D = F / heads;
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < A->n_rows; ++r)
        for (int32_t f = 0; f < F; ++f) dX[r * lddx + f] = dX[r * lddx + f] + d_aL[r * heads + f / D] * wR[f];
    return GALA_OK;
}

extern "C" int gala_cpu_head_attn_f32(int64_t n_rows, int32_t F, int32_t heads, const float *X, int64_t ldx,
                                      const float *w, const float *b, float *out, void *) {
    if (n_rows < 0 || F < 1 || heads < 1 || F % heads != 0 || ldx < F) return GALA_ERR_INVALID_ARG;
    if (n_rows == 0) return GALA_OK;
    if (!X || !w || !out) return GALA_ERR_INVALID_ARG;
    const int32_t D = F / heads;
#pragma omp parallel for schedule(static, 4096)
    for (int64_t r = 0; r < n_rows; ++r)
        for (int32_t h = 0; h < heads; ++h) {
            float acc = 0.0f;
            for (int32_t d = 0; d < D; ++d) acc = fmaf(X[r * ldx + h * D + d], w[h * D + d], acc);
            out[r * heads + h] = b ? acc + b[h] : acc;
        }
    return GALA_OK;
}

extern "C" int gala_cpu_head_attn_bwd_f32(int64_t n_rows, int32_t F, int32_t heads, const float *g,
                                          const float *w, float *dX, int64_t lddx, int32_t accumulate, void *) {
    if (n_rows < 0 || F < 1 || heads < 1 || F % heads != 0 || lddx < F) return GALA_ERR_INVALID_ARG;
    if (n_rows == 0) return GALA_OK;
    if (!g || !w || !dX) return GALA_ERR_INVALID_ARG;
    const int32_t D = F / heads;
#pragma omp parallel for schedule(static, 4096)
    for (int64_t r = 0; r < n_rows; ++r)
        for (int32_t c = 0; c < F; ++c) {
            const float m = g[r * heads + c / D] * w[c];
            dX[r * lddx + c] = accumulate ? dX[r * lddx + c] + m : m;
        }
    return GALA_OK;
}

extern "C" int gala_cpu_edge_permute_f32(const int32_t *perm, const float *src, int64_t n,
                                         int32_t heads, float *dst, void *) {
    if (n < 0 || heads < 1) return GALA_ERR_INVALID_ARG;
    if (n == 0) return GALA_OK;
    if (!perm || !src || !dst) return GALA_ERR_INVALID_ARG;
#pragma omp parallel for schedule(static, 4096)
    for (int64_t i = 0; i < n; ++i)
        for (int32_t h = 0; h < heads; ++h) dst[i * heads + h] = src[(int64_t)perm[i] * heads + h];
    return GALA_OK;
}

// FFN weight / bias gradients: fixed row chunks, per-chunk partial tiles, partials summed in
// chunk order (deterministic for given shapes, like the GPU kernel pair in dense.hip)
namespace {
constexpr int64_t kDenseChunk = 8192;
int64_t dense_chunks(int64_t n_rows) { return (n_rows + kDenseChunk - 1) / kDenseChunk; }
}  // namespace

extern "C" int64_t gala_cpu_dense_grad_workspace(int64_t n_rows, int32_t K, int32_t M) {
    if (n_rows < 0 || K < 0 || M < 0) return -1;
    if (n_rows == 0 || K == 0 || M == 0) return 0;
    return (int64_t)sizeof(float) * dense_chunks(n_rows) * ((int64_t)M * K + M);
}

extern "C" int gala_cpu_dense_grad_f32(int64_t n_rows, int32_t K, int32_t M, const float *X,
                                       int64_t ldx, const float *dY, int64_t ldy, float *dW,
                                       float *db, int32_t accumulate, void *workspace,
                                       int64_t workspace_bytes, void *) {
    if (n_rows < 0 || K < 0 || M < 0 || ldx < K || ldy < M) return GALA_ERR_INVALID_ARG;
    if (K == 0 || M == 0) return GALA_OK;
    if (!dW) return GALA_ERR_INVALID_ARG;
    const int64_t MK = (int64_t)M * K;
    if (n_rows == 0) {
        if (!accumulate) {
            std::fill(dW, dW + MK, 0.0f);
            if (db) std::fill(db, db + M, 0.0f);
        }
        return GALA_OK;
    }
    if (!X || !dY || !workspace) return GALA_ERR_INVALID_ARG;
    const int64_t P = dense_chunks(n_rows);
    if (workspace_bytes < (int64_t)sizeof(float) * P * (MK + M)) return GALA_ERR_INVALID_ARG;
    float *part = (float *)workspace;
    float *bpart = part + P * MK;
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t p = 0; p < P; ++p) {
        float *w = part + p * MK;
        float *b = bpart + p * M;
        std::fill(w, w + MK, 0.0f);
        std::fill(b, b + M, 0.0f);
        const int64_t r1 = std::min(n_rows, (p + 1) * kDenseChunk);
        for (int64_t n = p * kDenseChunk; n < r1; ++n) {
            const float *xr = X + n * ldx;
            for (int32_t m = 0; m < M; ++m) {
                const float y = dY[n * ldy + m];
                float *wm = w + (int64_t)m * K;
                for (int32_t k = 0; k < K; ++k) wm[k] = fmaf(y, xr[k], wm[k]);
                b[m] = b[m] + y;
            }
        }
    }
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < MK; ++i) {
        float s = 0.0f;
        for (int64_t p = 0; p < P; ++p) s = s + part[p * MK + i];
        dW[i] = accumulate ? dW[i] + s : s;
    }
    if (db)
        for (int32_t m = 0; m < M; ++m) {
            float s = 0.0f;
            for (int64_t p = 0; p < P; ++p) s = s + bpart[p * M + m];
            db[m] = accumulate ? db[m] + s : s;
        }
    return GALA_OK;
}

// ---- the multi-head GAT layer in input space (gala_gat_in_*, gat_input.hip) -------------
// The same extended rows and the same sums in the same order as the gfx950 kernels (the
// matrix cores' k-ordered fmaf chains: the edges of a row in CSR order; the projection over
// the feature tiles; the backward's column partials per persistent workgroup, summed in
// workgroup order); exp is the host's, so values agree to fp32 rounding.
namespace {

constexpr int kInLd = 128, kInMaxFin = 100, kInMaxHeads = 8, kInTiles = 7, kInWaves = 8, kInGrid = 512;
constexpr int kOnesSlot = 112;
inline int aR_slot(int h) { return 67 + 4 * h; }
inline int aL_slot(int h) { return 99 + 4 * h; }
inline int q_slot(int h) { return 116 + 4 * (h / 3) + h % 3; }
inline int tile_feature(int t, int m, int fin) {
    int f;
    if (t < 4) f = 4 * m + t;
    else if (m < 12) f = 64 + 3 * m + (t - 4);
    else return (m == 12 && t == 4) ? -2 : -1;
    return f < fin ? f : -1;
}
// extended-row slot of tile t's row m (the kernels' lane / component layout)
inline int tile_slot(int t, int m) { return t < 4 ? 4 * m + t : 64 + 4 * m + (t - 4); }

int check_in_graph(const gala_csr_t *A, int32_t fin, int32_t heads, int32_t D) {
    int st = check_csr(A);
    if (st) return st;
    if (fin < 1 || heads < 1 || D < 1) return GALA_ERR_INVALID_ARG;
    if (fin > kInMaxFin || heads > kInMaxHeads || !(D == 4 || D == 8 || D == 16 || D == 32) || A->n_seg != 1 ||
        A->n_rows != A->n_cols || (A->split && A->split->n_rows_split > 0))
        return GALA_ERR_UNSUPPORTED;
    return GALA_OK;
}

// the d_aL dots over D / 4 lanes of four features each, summed by the kernels' xor butterfly
float butterfly_dot(const float *a, const float *b, int D) {
    float v[8];
    const int L = D / 4;
    for (int l = 0; l < L; ++l) {
        float s = 0.0f;
        for (int i = 0; i < 4; ++i) s = fmaf(a[4 * l + i], b[4 * l + i], s);
        v[l] = s;
    }
    for (int o = L / 2; o >= 1; o /= 2) {
        float w[8];
        for (int l = 0; l < L; ++l) w[l] = v[l] + v[l ^ o];
        for (int l = 0; l < L; ++l) v[l] = w[l];
    }
    return v[0];
}

}  // namespace

extern "C" int gala_cpu_gat_in_prep_f32(int64_t n, int32_t fin, const float *Xin, int64_t ldxin, int32_t heads,
                                        const float *u, const float *c, float *Xext, void *stream) {
    (void)stream;
    if (n < 0 || fin < 1 || heads < 1 || ldxin < fin) return GALA_ERR_INVALID_ARG;
    if (fin > kInMaxFin || heads > kInMaxHeads) return GALA_ERR_UNSUPPORTED;
    if (n == 0) return GALA_OK;
    if (!Xin || !u || !c || !Xext) return GALA_ERR_INVALID_ARG;
    const int H = heads;
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < n; ++r) {
        const float *x = Xin + r * ldxin;
        float *o = Xext + r * kInLd;
        // the kernel's association: 16 lane partials (lane n: features 4n..4n+3, then
        // 64+3n..64+3n+2), summed by the xor butterfly 8, 4, 2, 1
        float lg[2 * kInMaxHeads] = {0.0f};
        for (int k = 0; k < 2 * H; ++k) {
            float v[16];
            for (int nn = 0; nn < 16; ++nn) {
                float d = 0.0f;
                for (int i = 0; i < 4; ++i) {
                    const int f = 4 * nn + i;
                    d = fmaf(f < fin ? x[f] : 0.0f, f < fin ? u[k * fin + f] : 0.0f, d);
                }
                for (int i = 0; i < 3; ++i) {
                    const int f = 64 + 3 * nn + i;
                    const bool ok = nn < 12 && f < fin;
                    d = fmaf(ok ? x[f] : 0.0f, ok ? u[k * fin + f] : 0.0f, d);
                }
                v[nn] = d;
            }
            for (int o = 8; o >= 1; o /= 2) {
                float w[16];
                for (int nn = 0; nn < 16; ++nn) w[nn] = v[nn] + v[nn ^ o];
                for (int nn = 0; nn < 16; ++nn) v[nn] = w[nn];
            }
            lg[k] = v[0];
        }
        for (int s = 0; s < kInLd; ++s) {
            float v = 0.0f;
            if (s < 64) {
                v = s < fin ? x[s] : 0.0f;
            } else {
                const int nn = (s - 64) >> 2, cc = (s - 64) & 3;
                if (cc < 3 && nn < 12) {
                    const int f = 64 + 3 * nn + cc;
                    v = f < fin ? x[f] : 0.0f;
                } else if (s == kOnesSlot) {
                    v = 1.0f;
                } else if (cc == 3 && nn < kInMaxHeads) {
                    v = nn < H ? lg[H + nn] + c[H + nn] : 0.0f;
                } else if (cc == 3) {
                    v = nn - 8 < H ? lg[nn - 8] + c[nn - 8] : 0.0f;
                }
            }
            o[s] = v;
        }
    }
    return GALA_OK;
}

extern "C" int gala_cpu_gat_in_fwd_f32(const gala_csr_t *A, const int32_t *order_in, int32_t fin, int32_t heads,
                                       int32_t D, float slope,
                                       float *Xext, const float *W, int64_t ldw, const float *b, float *Y,
                                       float *Ym, int64_t ldy, float *q, float *sma, int32_t flags, void *stream) {
    (void)stream;
    int st = check_in_graph(A, fin, heads, D);
    if (st) return st;
    if (ldw < fin || ldy < (int64_t)heads * D || (flags & ~GALA_GAT_IN_RELU)) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0) return GALA_OK;
    if (!Xext || !W || !Y || !Ym || !q || !sma) return GALA_ERR_INVALID_ARG;
    const bool relu = flags & GALA_GAT_IN_RELU;
    const int H = heads;
    const int32_t *order = order_in ? order_in : (A->split ? A->split->row_order : nullptr);
    std::vector<float> qv((size_t)A->n_rows * H);
#pragma omp parallel
    {
        std::vector<float> Z((size_t)16 * kInTiles * 16);   // [variant][tile][m]
#pragma omp for schedule(dynamic, kRowChunk)
        for (int64_t ri = 0; ri < A->n_rows; ++ri) {
            const int64_t r = order ? order[ri] : ri;
            std::fill(Z.begin(), Z.end(), 0.0f);
            const float *xr = Xext + r * kInLd;
            for (int64_t e = A->rowptr[r]; e < A->rowptr[r + 1]; ++e) {
                const float *xc = Xext + (int64_t)A->col[e] * kInLd;
                float pv[8], mp[8];
                for (int h = 0; h < 8; ++h) {
                    pv[h] = mp[h] = 0.0f;
                    if (h >= H) continue;
                    const float t = xr[aL_slot(h)] + xc[aR_slot(h)];
                    const bool pos = t > 0.0f;
                    pv[h] = ref_exp(pos ? t : t * slope);
                    mp[h] = pos ? pv[h] : pv[h] * slope;
                }
                for (int v = 0; v < 16; ++v) {
                    const float bv = v < 8 ? pv[v] : mp[v - 8];
                    for (int t = 0; t < kInTiles; ++t)
                        for (int m = 0; m < 16; ++m) {
                            const float a = (t >= 4 && m >= 13) ? 0.0f : xc[tile_slot(t, m)];
                            float &z = Z[((size_t)v * kInTiles + t) * 16 + m];
                            z = fmaf(a, bv, z);
                        }
                }
            }
            for (int h = 0; h < H; ++h) {
                const float S = Z[((size_t)h * kInTiles + 4) * 16 + 12];
                const float Sm = Z[((size_t)(h + 8) * kInTiles + 4) * 16 + 12];
                const float qq = 1.0f / (S + 1e-12f);
                for (int j = 0; j < D; ++j) {
                    float y0 = 0.0f, y1 = 0.0f;
                    const int64_t o = (int64_t)h * D + j;
                    for (int t = 0; t < kInTiles; ++t)
                        for (int q4 = 0; q4 < 4; ++q4)
                            for (int kq = 0; kq < 4; ++kq) {
                                const int m = 4 * kq + q4, f = tile_feature(t, m, fin);
                                const float w = f >= 0 ? W[o * ldw + f] : (f == -2 && b ? b[o] : 0.0f);
                                y0 = fmaf(Z[((size_t)h * kInTiles + t) * 16 + m], w, y0);
                                y1 = fmaf(Z[((size_t)(h + 8) * kInTiles + t) * 16 + m], w, y1);
                            }
                    const float yv = qq * y0;
                    Y[r * ldy + o] = (!relu || yv > 0.0f || yv != yv) ? yv : 0.0f;
                    Ym[r * ldy + o] = qq * y1;
                }
                q[r * H + h] = qq;
                qv[(size_t)r * H + h] = qq;
                sma[r * H + h] = qq * Sm;
            }
        }
    }
    // q into the extended rows after every row has read its neighbours' (as the kernels'
    // slots, which no aggregation reads)
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < A->n_rows; ++r)
        for (int h = 0; h < H; ++h) Xext[r * kInLd + q_slot(h)] = qv[(size_t)r * H + h];
    return GALA_OK;
}

extern "C" int64_t gala_cpu_gat_in_bwd_workspace(int32_t heads) {
    if (heads < 1 || heads > kInMaxHeads) return -1;
    return (int64_t)kInGrid * heads * 2 * kInTiles * 64 * 4 * (int64_t)sizeof(float);
}

extern "C" int gala_cpu_gat_in_bwd_f32(const gala_csr_t *AT, const int32_t *order_in, int32_t fin, int32_t heads,
                                       int32_t D, float slope,
                                       const float *Xext, const float *dY, const float *Y, const float *Ym,
                                       int64_t ldy, const float *sma, float *daL, float *M, void *ws,
                                       int64_t ws_bytes, int32_t flags, void *stream) {
    (void)stream;
    int st = check_in_graph(AT, fin, heads, D);
    if (st) return st;
    if (ldy < (int64_t)heads * D || (ldy & 3) || (flags & ~GALA_GAT_IN_RELU)) return GALA_ERR_INVALID_ARG;
    if (!M) return GALA_ERR_INVALID_ARG;
    const int H = heads;
    const bool relu = flags & GALA_GAT_IN_RELU;
    const int64_t outn = (int64_t)H * D * (fin + 1);
    std::fill(M, M + outn, 0.0f);
    if (AT->n_rows == 0) return GALA_OK;
    if (!Xext || !dY || !Y || !Ym || !sma || !daL || !ws) return GALA_ERR_INVALID_ARG;
    if (ws_bytes < gala_cpu_gat_in_bwd_workspace(heads)) return GALA_ERR_INVALID_ARG;
    const int32_t *order = order_in ? order_in : (AT->split ? AT->split->row_order : nullptr);
    const int64_t n = AT->n_rows, nblk = (n + kInWaves - 1) / kInWaves;
    const int grid = (int)std::min<int64_t>(std::max<int64_t>(nblk, 1), kInGrid);
    const int64_t per = (int64_t)H * D * (fin + 1);
    float *part = (float *)ws;   // [grid][H][D][fin + 1]
    const int F = H * D;
#pragma omp parallel
    {
        std::vector<float> T((size_t)kInMaxHeads * kInTiles * 16);
#pragma omp for schedule(dynamic, 1)
        for (int g = 0; g < grid; ++g) {
            float *Mg = part + (int64_t)g * per;
            std::fill(Mg, Mg + per, 0.0f);
            for (int64_t blk = g; blk < nblk; blk += grid)
                for (int w = 0; w < kInWaves; ++w) {
                    const int64_t ci = blk * kInWaves + w;
                    if (ci >= n) break;
                    const int64_t c = order ? order[ci] : ci;
                    std::fill(T.begin(), T.end(), 0.0f);
                    const float *xc = Xext + c * kInLd;
                    for (int64_t e = AT->rowptr[c]; e < AT->rowptr[c + 1]; ++e) {
                        const float *xr = Xext + (int64_t)AT->col[e] * kInLd;
                        for (int h = 0; h < H; ++h) {
                            const float t = xr[aL_slot(h)] + xc[aR_slot(h)];
                            const float a = ref_exp(t > 0.0f ? t : t * slope) * xr[q_slot(h)];
                            for (int tt = 0; tt < kInTiles; ++tt)
                                for (int m = 0; m < 16; ++m) {
                                    const float x = (tt >= 4 && m >= 13) ? 0.0f : xr[tile_slot(tt, m)];
                                    float &z = T[((size_t)h * kInTiles + tt) * 16 + m];
                                    z = fmaf(x, a, z);
                                }
                        }
                    }
                    for (int h = 0; h < H; ++h) {
                        float dym[32];   // dY, masked by relu(Y) > 0 with the fused ReLU
                        const float *yh = Y + c * ldy + (int64_t)h * D;
                        for (int j = 0; j < D; ++j) dym[j] = (!relu || yh[j] > 0.0f) ? dY[c * ldy + (int64_t)h * D + j] : 0.0f;
                        const float *dy = dym;
                        const float sy = butterfly_dot(dy, Y + c * ldy + (int64_t)h * D, D);
                        const float sm = butterfly_dot(dy, Ym + c * ldy + (int64_t)h * D, D);
                        const float accv = sy + 1e-12f;
                        daL[c * H + h] = (sm - accv * sma[c * H + h]) + 1e-12f;
                        for (int j = 0; j < D; ++j)
                            for (int tt = 0; tt < kInTiles; ++tt)
                                for (int m = 0; m < 16; ++m) {
                                    const int f = tile_feature(tt, m, fin);
                                    if (f == -1) continue;
                                    float &z = Mg[((int64_t)h * D + j) * (fin + 1) + (f == -2 ? fin : f)];
                                    z = fmaf(dy[j], T[((size_t)h * kInTiles + tt) * 16 + m], z);
                                }
                    }
                }
        }
    }
    (void)F;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < per; ++i) {
        float s = 0.0f;
        for (int g = 0; g < grid; ++g) s += part[(int64_t)g * per + i];
        M[i] = s;
    }
    return GALA_OK;
}
