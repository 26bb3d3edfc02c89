// Edge-parallel ops of the GAT pipeline for gfx950: SDDVV (add / mul / add+LeakyReLU),
// edge->row sum, row->edge scale, SDDMM dot, edge-softmax forward/backward, the fused
// GAT aggregation and the edge-value permutation.
//
// Replaces the emitted kernels default_function_kernel_sddvv_{plus,mult}_undir
// (src/codegen/cuda.h:679-698, 848-867), spmm_backward_sddmm_32_{nln,eaggr}
// (505-524, 659-678), {softmax,mult}_sddvv_undir (525-562), sddmm_mult_undir_shared
// (699-734) and the torch compositions around them (src/codegen/common.h:735-810).
//
// Row-segment ops ("RS" kernels): a group of G lanes owns one row and strides over its
// edges (coalesced edge arrays), reductions use xor butterflies inside the group.
#include "gala_internal.h"

namespace gala {

struct EdgeParams {
    const int32_t *rowptr;
    const int32_t *col;
    int64_t n_rows;
    int32_t heads;
    SegTable seg;
};

__device__ __forceinline__ void row_range(const EdgeParams &p, int s, int64_t row, int64_t &e0,
                                          int64_t &e1) {
    const int32_t *rp = p.rowptr + (int64_t)p.seg.rp[s] * (p.n_rows + 1);
    e0 = (int64_t)p.seg.base[s] + rp[row];
    e1 = (int64_t)p.seg.base[s] + rp[row + 1];
}

#define GALA_ROW_PROLOGUE(G)                                                          \
    const int lane = threadIdx.x & (kWave - 1);                                       \
    const int gl = lane & ((G)-1);                                                    \
    const int64_t row = ((int64_t)blockIdx.x * (kBlock / kWave) + threadIdx.x / kWave) \
                            * (kWave / (G)) + lane / (G);                             \
    const bool row_ok = row < p.n_rows;

// ---- SDDVV --------------------------------------------------------------------------
template <int G, int OP>
__global__ __launch_bounds__(kBlock) void k_sddvv(EdgeParams p, const float *a, const float *b,
                                                  float slope, float *out) {
    GALA_ROW_PROLOGUE(G);
    if (!row_ok) return;
    const int H = p.heads;
    for (int s = 0; s < p.seg.n; ++s) {
        int64_t e0, e1;
        row_range(p, s, row, e0, e1);
        const int64_t n = (e1 - e0) * H;
        for (int64_t t = gl; t < n; t += G) {
            const int64_t e = e0 + t / H;
            const int h = (int)(t % H);
            const float av = a[row * H + h];
            const float bv = b[(int64_t)p.col[e] * H + h];
            float r;
            if (OP == GALA_SDDVV_MUL) {
                r = __fmul_rn(av, bv);
            } else {
                r = __fadd_rn(av, bv);
                if (OP == GALA_SDDVV_ADD_LRELU) r = r > 0.0f ? r : __fmul_rn(r, slope);
            }
            out[e * H + h] = r;
        }
    }
}

// ---- edge -> row sum (K7) ----------------------------------------------------------
template <int G>
__global__ __launch_bounds__(kBlock) void k_row_sum(EdgeParams p, const float *v, float eps,
                                                    int accum, float *out) {
    GALA_ROW_PROLOGUE(G);
    const int H = p.heads;
    for (int h = 0; h < H; ++h) {
        float part = 0.0f;
        if (row_ok) {
            for (int s = 0; s < p.seg.n; ++s) {
                int64_t e0, e1;
                row_range(p, s, row, e0, e1);
                for (int64_t e = e0 + gl; e < e1; e += G) part += v[e * H + h];
            }
        }
        part = group_sum<G>(part);
        if (row_ok && gl == 0) {
            // reference: each segment's sum starts at 1e-12 (cuda.h:512,666)
            float r = part + (float)p.seg.n * eps;
            if (accum) r = out[row * H + h] + r;
            out[row * H + h] = r;
        }
    }
}

// ---- row -> edge scale (K8) --------------------------------------------------------
template <int G>
__global__ __launch_bounds__(kBlock) void k_row_scale(EdgeParams p, const float *q, float *v) {
    GALA_ROW_PROLOGUE(G);
    if (!row_ok) return;
    const int H = p.heads;
    for (int s = 0; s < p.seg.n; ++s) {
        int64_t e0, e1;
        row_range(p, s, row, e0, e1);
        const int64_t n = (e1 - e0) * H;
        for (int64_t t = gl; t < n; t += G) {
            const int64_t idx = e0 * H + t;
            v[idx] = __fmul_rn(v[idx], q[row * H + (int)(t % H)]);
        }
    }
}

// ---- edge softmax -------------------------------------------------------------------
__device__ __forceinline__ float ref_exp(float s) {
    // torch::exp then torch::clamp(0, 1e12) (common.h:760-761); NaN propagates like clamp
    const float p = expf(s);
    return p > 1e12f ? 1e12f : p;
}

template <int G, int MODE>
__global__ __launch_bounds__(kBlock) void k_softmax_fwd(EdgeParams p, const float *logit,
                                                        float *alpha) {
    GALA_ROW_PROLOGUE(G);
    const int H = p.heads;
    for (int h = 0; h < H; ++h) {
        float m = -INFINITY, sum = 0.0f;
        if (row_ok) {
            for (int s = 0; s < p.seg.n; ++s) {
                int64_t e0, e1;
                row_range(p, s, row, e0, e1);
                for (int64_t e = e0 + gl; e < e1; e += G) {
                    const float x = logit[e * H + h];
                    if (MODE == GALA_SOFTMAX_REF) {
                        sum += ref_exp(x);
                    } else {  // online max/sum
                        if (x > m) {
                            sum = sum * expf(m - x) + 1.0f;
                            m = x;
                        } else {
                            sum += expf(x - m);
                        }
                    }
                }
            }
        }
        float q;
        if (MODE == GALA_SOFTMAX_REF) {
            sum = group_sum<G>(sum);
            q = 1.0f / (sum + (float)p.seg.n * 1e-12f);  // torch::reciprocal(row_sum)
        } else {
            const float gm = group_max<G>(m);
            sum = (m == -INFINITY) ? 0.0f : sum * expf(m - gm);
            sum = group_sum<G>(sum);
            m = gm;
            q = 1.0f / sum;
        }
        if (!row_ok) continue;
        for (int s = 0; s < p.seg.n; ++s) {
            int64_t e0, e1;
            row_range(p, s, row, e0, e1);
            for (int64_t e = e0 + gl; e < e1; e += G) {
                const float x = logit[e * H + h];
                const float pe = (MODE == GALA_SOFTMAX_REF) ? ref_exp(x) : expf(x - m);
                alpha[e * H + h] = __fmul_rn(pe, q);
            }
        }
    }
}

template <int G, int MODE>
__global__ __launch_bounds__(kBlock) void k_softmax_bwd(EdgeParams p, const float *alpha,
                                                        const float *dalpha, float *dlogit) {
    GALA_ROW_PROLOGUE(G);
    const int H = p.heads;
    const float eps = (MODE == GALA_SOFTMAX_REF) ? 1e-12f : 0.0f;
    for (int h = 0; h < H; ++h) {
        float part = 0.0f;
        if (row_ok) {
            for (int s = 0; s < p.seg.n; ++s) {
                int64_t e0, e1;
                row_range(p, s, row, e0, e1);
                for (int64_t e = e0 + gl; e < e1; e += G)
                    part += __fmul_rn(alpha[e * H + h], dalpha[e * H + h]);
            }
        }
        part = group_sum<G>(part);
        const float acc = part + (float)p.seg.n * eps;  // K7 on sds (common.h:793-794)
        if (!row_ok) continue;
        for (int s = 0; s < p.seg.n; ++s) {
            int64_t e0, e1;
            row_range(p, s, row, e0, e1);
            for (int64_t e = e0 + gl; e < e1; e += G) {
                const float a = alpha[e * H + h];
                const float sds = __fmul_rn(a, dalpha[e * H + h]);
                dlogit[e * H + h] = __fsub_rn(sds, __fmul_rn(a, acc));  // sds - K8(acc)
            }
        }
    }
}

// ---- SDDMM dot (K9) -----------------------------------------------------------------
// Row group of G lanes over the features (VEC per lane), heads reduce over HW lanes.
template <int G, int VEC, int HW>
__global__ __launch_bounds__(kBlock) void k_sddmm(EdgeParams p, const float *Ad, int64_t lda,
                                                  const float *Bd, int64_t ldb, int32_t F,
                                                  float *out) {
    GALA_ROW_PROLOGUE(G);
    const int f = gl * VEC;
    const bool cv = row_ok && f < F;
    float a[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) a[i] = cv ? Ad[row * lda + f + i] : 0.0f;
    const int H = p.heads;
    const int D = F / H;
    const int h = cv ? f / D : 0;
    // wave-uniform loop bound: groups of one wave own different rows
    for (int s = 0; s < p.seg.n; ++s) {
        int64_t e0 = 0, e1 = 0;
        if (row_ok) row_range(p, s, row, e0, e1);
        const int64_t n = e1 - e0;
        int64_t nmax = n;
#pragma unroll
        for (int o = 32; o >= G; o >>= 1) {
            const int64_t other = __shfl_xor((long long)nmax, o, 64);
            nmax = other > nmax ? other : nmax;
        }
        for (int64_t j = 0; j < nmax; ++j) {
            float part = 0.0f;
            if (j < n && cv) {
                const int64_t c = p.col[e0 + j];
                const float *bp = Bd + c * ldb + f;
#pragma unroll
                for (int i = 0; i < VEC; ++i) part = fmaf(a[i], bp[i], part);
            }
            part = group_sum<HW>(part);
            if (j < n && cv && (gl % HW) == 0) out[(e0 + j) * H + h] = part;
        }
    }
}

// ---- fused GAT aggregation -----------------------------------------------------------
// Row group of G lanes over the F = heads*D features (one feature per lane per chunk).
template <int G, int CH, int MODE>
__global__ __launch_bounds__(kBlock) void k_gat_fwd(EdgeParams p, const float *aL, const float *aR,
                                                    const float *X, int64_t ldx, int32_t F,
                                                    float slope, float *Y, int64_t ldy,
                                                    float *alpha_out) {
    GALA_ROW_PROLOGUE(G);
    if (!row_ok) return;
    const int H = p.heads;
    const int D = F / H;
    float acc[CH], m[CH], sum[CH], al[CH];
    int hh[CH];
    bool cv[CH];
#pragma unroll
    for (int ch = 0; ch < CH; ++ch) {
        const int f = ch * G + gl;
        cv[ch] = f < F;
        hh[ch] = cv[ch] ? f / D : 0;
        acc[ch] = 0.0f;
        m[ch] = -INFINITY;
        sum[ch] = 0.0f;
        al[ch] = aL[row * H + hh[ch]];
    }
    for (int s = 0; s < p.seg.n; ++s) {
        int64_t e0, e1;
        row_range(p, s, row, e0, e1);
        for (int64_t e = e0; e < e1; ++e) {
            const int64_t c = p.col[e];
#pragma unroll
            for (int ch = 0; ch < CH; ++ch) {
                if (!cv[ch]) continue;
                float z = __fadd_rn(al[ch], aR[c * H + hh[ch]]);
                z = z > 0.0f ? z : __fmul_rn(z, slope);
                const float x = X[c * ldx + ch * G + gl];
                if (MODE == GALA_SOFTMAX_REF) {
                    const float pe = ref_exp(z);
                    sum[ch] = __fadd_rn(sum[ch], pe);
                    acc[ch] = fmaf(pe, x, acc[ch]);
                } else {
                    if (z > m[ch]) {
                        const float r = expf(m[ch] - z);
                        sum[ch] = fmaf(sum[ch], r, 1.0f);
                        acc[ch] = fmaf(acc[ch], r, x);
                        m[ch] = z;
                    } else {
                        const float pe = expf(z - m[ch]);
                        sum[ch] = __fadd_rn(sum[ch], pe);
                        acc[ch] = fmaf(pe, x, acc[ch]);
                    }
                }
            }
        }
    }
    float q[CH];
#pragma unroll
    for (int ch = 0; ch < CH; ++ch) {
        if (!cv[ch]) continue;
        const float den = (MODE == GALA_SOFTMAX_REF) ? sum[ch] + (float)p.seg.n * 1e-12f : sum[ch];
        q[ch] = 1.0f / den;
        Y[row * ldy + ch * G + gl] = (sum[ch] == 0.0f && MODE != GALA_SOFTMAX_REF)
                                         ? 0.0f
                                         : __fmul_rn(acc[ch], q[ch]);
    }
    if (alpha_out) {
        // one lane per head writes alpha (lane holding the head's first feature)
        for (int s = 0; s < p.seg.n; ++s) {
            int64_t e0, e1;
            row_range(p, s, row, e0, e1);
            for (int64_t e = e0; e < e1; ++e) {
                const int64_t c = p.col[e];
#pragma unroll
                for (int ch = 0; ch < CH; ++ch) {
                    const int f = ch * G + gl;
                    if (!cv[ch] || (f % D) != 0) continue;
                    float z = __fadd_rn(al[ch], aR[c * H + hh[ch]]);
                    z = z > 0.0f ? z : __fmul_rn(z, slope);
                    const float pe = (MODE == GALA_SOFTMAX_REF) ? ref_exp(z) : expf(z - m[ch]);
                    alpha_out[e * H + hh[ch]] = __fmul_rn(pe, q[ch]);
                }
            }
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_permute(const int32_t *perm, const float *src,
                                                    int64_t n, int32_t H, float *dst) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= n * H) return;
    const int64_t i = t / H;
    const int h = (int)(t % H);
    dst[t] = src[(int64_t)perm[i] * H + h];
}

// ---- host side ------------------------------------------------------------------------
static int pick_group(const gala_csr_t *A, int heads) {
    // lanes per row from the mean row length (edges*heads)
    const double avg = A->n_rows ? (double)A->nnz * heads / (double)A->n_rows : 1.0;
    int g = 4;
    while (g < 64 && g < avg) g <<= 1;
    return g;
}

static int edge_setup(const gala_csr_t *A, int32_t heads, EdgeParams *p) {
    int st = check_csr(A);
    if (st) return st;
    if (heads < 1) return GALA_ERR_INVALID_ARG;
    if (A->n_seg > kMaxSegPerLaunch) return GALA_ERR_UNSUPPORTED;
    p->rowptr = A->rowptr;
    p->col = A->col;
    p->n_rows = A->n_rows;
    p->heads = heads;
    return fill_segments(A, 0, &p->seg);
}

static unsigned blocks_for(int64_t n_rows, int G) {
    const int64_t rpb = (int64_t)(kBlock / kWave) * (kWave / G);
    return (unsigned)((n_rows + rpb - 1) / rpb);
}

#define GALA_DISPATCH_G(G, ...)                        \
    switch (G) {                                       \
        case 4: { constexpr int GG = 4; __VA_ARGS__; } break;   \
        case 8: { constexpr int GG = 8; __VA_ARGS__; } break;   \
        case 16: { constexpr int GG = 16; __VA_ARGS__; } break; \
        case 32: { constexpr int GG = 32; __VA_ARGS__; } break; \
        default: { constexpr int GG = 64; __VA_ARGS__; } break; \
    }

}  // namespace gala

using namespace gala;

extern "C" int gala_sddvv_f32(const gala_csr_t *A, const float *a_row, const float *b_col,
                              int32_t heads, int32_t op, float slope, float *out_e,
                              void *stream) {
    EdgeParams p;
    int st = edge_setup(A, heads, &p);
    if (st) return st;
    if (op < GALA_SDDVV_ADD || op > GALA_SDDVV_ADD_LRELU) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0 || A->nnz == 0) return GALA_OK;
    if (!a_row || !b_col || !out_e) return GALA_ERR_INVALID_ARG;
    const int G = pick_group(A, heads);
    hipStream_t hs = (hipStream_t)stream;
    GALA_DISPATCH_G(G, {
        if (op == GALA_SDDVV_ADD)
            hipLaunchKernelGGL((k_sddvv<GG, GALA_SDDVV_ADD>), dim3(blocks_for(A->n_rows, GG)),
                               dim3(kBlock), 0, hs, p, a_row, b_col, slope, out_e);
        else if (op == GALA_SDDVV_MUL)
            hipLaunchKernelGGL((k_sddvv<GG, GALA_SDDVV_MUL>), dim3(blocks_for(A->n_rows, GG)),
                               dim3(kBlock), 0, hs, p, a_row, b_col, slope, out_e);
        else
            hipLaunchKernelGGL((k_sddvv<GG, GALA_SDDVV_ADD_LRELU>),
                               dim3(blocks_for(A->n_rows, GG)), dim3(kBlock), 0, hs, p, a_row,
                               b_col, slope, out_e);
    });
    return launch_status();
}

extern "C" int gala_row_sum_f32(const gala_csr_t *A, const float *v_e, int32_t heads, float eps,
                                float *out_row, int32_t flags, void *stream) {
    EdgeParams p;
    int st = edge_setup(A, heads, &p);
    if (st) return st;
    if (flags & ~GALA_SPMM_ACCUM) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0) return GALA_OK;
    if (!out_row || (!v_e && A->nnz > 0)) return GALA_ERR_INVALID_ARG;
    const int G = pick_group(A, 1);
    const int accum = (flags & GALA_SPMM_ACCUM) ? 1 : 0;
    GALA_DISPATCH_G(G, hipLaunchKernelGGL((k_row_sum<GG>), dim3(blocks_for(A->n_rows, GG)),
                                          dim3(kBlock), 0, (hipStream_t)stream, p, v_e, eps,
                                          accum, out_row));
    return launch_status();
}

extern "C" int gala_row_scale_f32(const gala_csr_t *A, const float *q_row, int32_t heads,
                                  float *v_inout, void *stream) {
    EdgeParams p;
    int st = edge_setup(A, heads, &p);
    if (st) return st;
    if (A->n_rows == 0 || A->nnz == 0) return GALA_OK;
    if (!q_row || !v_inout) return GALA_ERR_INVALID_ARG;
    const int G = pick_group(A, heads);
    GALA_DISPATCH_G(G, hipLaunchKernelGGL((k_row_scale<GG>), dim3(blocks_for(A->n_rows, GG)),
                                          dim3(kBlock), 0, (hipStream_t)stream, p, q_row,
                                          v_inout));
    return launch_status();
}

extern "C" int gala_edge_softmax_fwd_f32(const gala_csr_t *A, const float *logits,
                                         int32_t heads, int32_t mode, float *alpha,
                                         void *stream) {
    EdgeParams p;
    int st = edge_setup(A, heads, &p);
    if (st) return st;
    if (mode != GALA_SOFTMAX_REF && mode != GALA_SOFTMAX_FIXED) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0 || A->nnz == 0) return GALA_OK;
    if (!logits || !alpha) return GALA_ERR_INVALID_ARG;
    const int G = pick_group(A, 1);
    hipStream_t hs = (hipStream_t)stream;
    GALA_DISPATCH_G(G, {
        if (mode == GALA_SOFTMAX_REF)
            hipLaunchKernelGGL((k_softmax_fwd<GG, GALA_SOFTMAX_REF>),
                               dim3(blocks_for(A->n_rows, GG)), dim3(kBlock), 0, hs, p, logits,
                               alpha);
        else
            hipLaunchKernelGGL((k_softmax_fwd<GG, GALA_SOFTMAX_FIXED>),
                               dim3(blocks_for(A->n_rows, GG)), dim3(kBlock), 0, hs, p, logits,
                               alpha);
    });
    return launch_status();
}

extern "C" int gala_edge_softmax_bwd_f32(const gala_csr_t *A, const float *alpha,
                                         const float *d_alpha, int32_t heads, int32_t mode,
                                         float *d_logits, void *stream) {
    EdgeParams p;
    int st = edge_setup(A, heads, &p);
    if (st) return st;
    if (mode != GALA_SOFTMAX_REF && mode != GALA_SOFTMAX_FIXED) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0 || A->nnz == 0) return GALA_OK;
    if (!alpha || !d_alpha || !d_logits) return GALA_ERR_INVALID_ARG;
    const int G = pick_group(A, 1);
    hipStream_t hs = (hipStream_t)stream;
    GALA_DISPATCH_G(G, {
        if (mode == GALA_SOFTMAX_REF)
            hipLaunchKernelGGL((k_softmax_bwd<GG, GALA_SOFTMAX_REF>),
                               dim3(blocks_for(A->n_rows, GG)), dim3(kBlock), 0, hs, p, alpha,
                               d_alpha, d_logits);
        else
            hipLaunchKernelGGL((k_softmax_bwd<GG, GALA_SOFTMAX_FIXED>),
                               dim3(blocks_for(A->n_rows, GG)), dim3(kBlock), 0, hs, p, alpha,
                               d_alpha, d_logits);
    });
    return launch_status();
}

template <int G, int VEC>
static void launch_sddmm(const EdgeParams &p, int hw, const float *Ad, int64_t lda,
                         const float *Bd, int64_t ldb, int32_t F, float *out, hipStream_t hs) {
    const dim3 grid(blocks_for(p.n_rows, G));
    switch (hw) {
        case 1: hipLaunchKernelGGL((k_sddmm<G, VEC, 1>), grid, dim3(kBlock), 0, hs, p, Ad, lda, Bd, ldb, F, out); break;
        case 2: hipLaunchKernelGGL((k_sddmm<G, VEC, (G < 2 ? G : 2)>), grid, dim3(kBlock), 0, hs, p, Ad, lda, Bd, ldb, F, out); break;
        case 4: hipLaunchKernelGGL((k_sddmm<G, VEC, (G < 4 ? G : 4)>), grid, dim3(kBlock), 0, hs, p, Ad, lda, Bd, ldb, F, out); break;
        case 8: hipLaunchKernelGGL((k_sddmm<G, VEC, (G < 8 ? G : 8)>), grid, dim3(kBlock), 0, hs, p, Ad, lda, Bd, ldb, F, out); break;
        case 16: hipLaunchKernelGGL((k_sddmm<G, VEC, (G < 16 ? G : 16)>), grid, dim3(kBlock), 0, hs, p, Ad, lda, Bd, ldb, F, out); break;
        case 32: hipLaunchKernelGGL((k_sddmm<G, VEC, (G < 32 ? G : 32)>), grid, dim3(kBlock), 0, hs, p, Ad, lda, Bd, ldb, F, out); break;
        default: hipLaunchKernelGGL((k_sddmm<G, VEC, G>), grid, dim3(kBlock), 0, hs, p, Ad, lda, Bd, ldb, F, out); break;
    }
}

template <int VEC>
static int sddmm_vec(const EdgeParams &p, int L, int hw, const float *Ad, int64_t lda,
                     const float *Bd, int64_t ldb, int32_t F, float *out, hipStream_t hs) {
    if (L <= 1) launch_sddmm<1, VEC>(p, hw, Ad, lda, Bd, ldb, F, out, hs);
    else if (L <= 2) launch_sddmm<2, VEC>(p, hw, Ad, lda, Bd, ldb, F, out, hs);
    else if (L <= 4) launch_sddmm<4, VEC>(p, hw, Ad, lda, Bd, ldb, F, out, hs);
    else if (L <= 8) launch_sddmm<8, VEC>(p, hw, Ad, lda, Bd, ldb, F, out, hs);
    else if (L <= 16) launch_sddmm<16, VEC>(p, hw, Ad, lda, Bd, ldb, F, out, hs);
    else if (L <= 32) launch_sddmm<32, VEC>(p, hw, Ad, lda, Bd, ldb, F, out, hs);
    else if (L <= 64) launch_sddmm<64, VEC>(p, hw, Ad, lda, Bd, ldb, F, out, hs);
    else return GALA_ERR_UNSUPPORTED;
    return GALA_OK;
}

extern "C" int gala_sddmm_dot_f32(const gala_csr_t *A, const float *Ad, int64_t lda,
                                  const float *Bd, int64_t ldb, int32_t F, int32_t heads,
                                  float *out_e, void *stream) {
    EdgeParams p;
    int st = edge_setup(A, heads, &p);
    if (st) return st;
    if (F < 1 || F % heads != 0 || lda < F || ldb < F) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0 || A->nnz == 0) return GALA_OK;
    if (!Ad || !Bd || !out_e) return GALA_ERR_INVALID_ARG;
    const int D = F / heads;
    // VEC divides D, L = lanes per row, the per-head lane count D/VEC must be a power of 2
    int vec = 4;
    while (vec > 1 && (D % vec || lda % vec || ldb % vec)) vec >>= 1;
    const int L = (F + vec - 1) / vec;
    const int hw_l = D / vec;
    int Gp = 1;
    while (Gp < L) Gp <<= 1;
    if (heads > 1 && (hw_l & (hw_l - 1))) return GALA_ERR_UNSUPPORTED;
    const int hw = heads > 1 ? hw_l : Gp;
    int r;
    if (vec == 4) r = sddmm_vec<4>(p, L, hw, Ad, lda, Bd, ldb, F, out_e, (hipStream_t)stream);
    else if (vec == 2) r = sddmm_vec<2>(p, L, hw, Ad, lda, Bd, ldb, F, out_e, (hipStream_t)stream);
    else r = sddmm_vec<1>(p, L, hw, Ad, lda, Bd, ldb, F, out_e, (hipStream_t)stream);
    if (r) return r;
    return launch_status();
}

template <int G, int CH>
static void launch_gat(const EdgeParams &p, int mode, const float *aL, const float *aR,
                       const float *X, int64_t ldx, int32_t F, float slope, float *Y,
                       int64_t ldy, float *alpha_out, hipStream_t hs) {
    const dim3 grid(blocks_for(p.n_rows, G));
    if (mode == GALA_SOFTMAX_REF)
        hipLaunchKernelGGL((k_gat_fwd<G, CH, GALA_SOFTMAX_REF>), grid, dim3(kBlock), 0, hs, p, aL,
                           aR, X, ldx, F, slope, Y, ldy, alpha_out);
    else
        hipLaunchKernelGGL((k_gat_fwd<G, CH, GALA_SOFTMAX_FIXED>), grid, dim3(kBlock), 0, hs, p,
                           aL, aR, X, ldx, F, slope, Y, ldy, alpha_out);
}

extern "C" int gala_gat_fwd_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                const float *X, int64_t ldx, int32_t F, int32_t heads,
                                float slope, int32_t mode, float *Y, int64_t ldy,
                                float *alpha_out, void *stream) {
    EdgeParams p;
    int st = edge_setup(A, heads, &p);
    if (st) return st;
    if (mode != GALA_SOFTMAX_REF && mode != GALA_SOFTMAX_FIXED) return GALA_ERR_INVALID_ARG;
    if (F < 1 || F % heads != 0 || ldx < F || ldy < F) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0) return GALA_OK;
    if (!aL || !aR || !Y || (!X && A->nnz > 0)) return GALA_ERR_INVALID_ARG;
    hipStream_t hs = (hipStream_t)stream;
    if (F <= 1) launch_gat<1, 1>(p, mode, aL, aR, X, ldx, F, slope, Y, ldy, alpha_out, hs);
    else if (F <= 2) launch_gat<2, 1>(p, mode, aL, aR, X, ldx, F, slope, Y, ldy, alpha_out, hs);
    else if (F <= 4) launch_gat<4, 1>(p, mode, aL, aR, X, ldx, F, slope, Y, ldy, alpha_out, hs);
    else if (F <= 8) launch_gat<8, 1>(p, mode, aL, aR, X, ldx, F, slope, Y, ldy, alpha_out, hs);
    else if (F <= 16) launch_gat<16, 1>(p, mode, aL, aR, X, ldx, F, slope, Y, ldy, alpha_out, hs);
    else if (F <= 32) launch_gat<32, 1>(p, mode, aL, aR, X, ldx, F, slope, Y, ldy, alpha_out, hs);
    else if (F <= 64) launch_gat<64, 1>(p, mode, aL, aR, X, ldx, F, slope, Y, ldy, alpha_out, hs);
    else if (F <= 128) launch_gat<64, 2>(p, mode, aL, aR, X, ldx, F, slope, Y, ldy, alpha_out, hs);
    else if (F <= 256) launch_gat<64, 4>(p, mode, aL, aR, X, ldx, F, slope, Y, ldy, alpha_out, hs);
    else if (F <= 512) launch_gat<64, 8>(p, mode, aL, aR, X, ldx, F, slope, Y, ldy, alpha_out, hs);
    else return GALA_ERR_UNSUPPORTED;
    return launch_status();
}

extern "C" int gala_edge_permute_f32(const int32_t *perm, const float *src, int64_t n,
                                     int32_t heads, float *dst, void *stream) {
    if (n < 0 || heads < 1) return GALA_ERR_INVALID_ARG;
    if (n == 0) return GALA_OK;
    if (!perm || !src || !dst) return GALA_ERR_INVALID_ARG;
    const int64_t total = n * heads;
    const int64_t blocks = (total + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(k_permute, dim3((unsigned)blocks), dim3(kBlock), 0, (hipStream_t)stream,
                       perm, src, n, heads, dst);
    return launch_status();
}
