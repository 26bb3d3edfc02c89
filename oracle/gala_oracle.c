/*
 * gala_oracle.c — TEST INFRASTRUCTURE ONLY (the parity oracle and the CPU baseline).
 *
 * Plain-C restatement of the reference's hot-path semantics, one function per
 * reference routine, each citing the reference file:line it follows.  It is linked
 * only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg; the product
 * library (libgala_hip.so) never calls it.
 *
 * Pinning: the layout builders and the SpMM are checked bit-for-bit against the
 * reference's own CPU code compiled from /root/reference (oracle/ref_harness.cpp ->
 * oracle/_ref/libgala_ref.so) through the committed fixtures in tests/golden/
 * (tests/test_oracle_golden.py).  The GPU-only kernels (SDDVV/SDDMM/row-sum/row-scale,
 * softmax compositions) have no CPU implementation in the reference; they are
 * restated line by line from the CUDA kernel strings (src/codegen/cuda.h) and the
 * torch compositions (src/codegen/common.h) and cross-checked against an independent
 * torch-CPU formulation in the tests.
 *
 * Rounding: compiled with -ffp-contract=off; fmaf() is written exactly where nvcc
 * contracts the reference's `a + b*c` (the emitted kernels), plain operations
 * elsewhere.  Edge order inside a row is the reference's CSR order.
 *
 * Graph arguments: rowptr holds n_seg blocks of (n_rows+1) relative offsets and
 * seg_base[s] is segment s's first edge (ord_col_tiling_torch layout, tiling.h:222-283);
 * n_seg == 1 with seg_base == NULL is a plain CSR.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define SEG_BASE(s) (seg_base ? (int64_t)seg_base[s] : 0)
#define ROWPTR(s) (rowptr + (int64_t)(s) * (n_rows + 1))

/* ---- SpMM: emitted aggregate_node_mul_sum*_kernel{k}[_offset] (cuda.h:286-436) ------
 * Per row: local = C[row, f] (C zero-filled by the wrapper, cuda.h:463, unless accum),
 * then for every segment launch (cuda.h:473-499, in segment order) and every edge j of
 * the row in CSR order: local = local + [A_e *] B[col_e, f]  (fma when weighted).
 * Kernel sampling (cuda.h:313-321): rows with jmax>0 take nsamp edges
 * j = (ra*ji + rb) % jmax.  src_scale/dst_scale restate the torch `norm * res`
 * broadcasts around the call (codegen/gala.cu:442-456): product rounded first. */
void orc_spmm(int64_t n_rows, int32_t n_seg, const int32_t *rowptr, const int32_t *seg_base,
              const int32_t *col, const float *val, int32_t val_heads, const float *X,
              int64_t ldx, int32_t F, const float *src_scale, const float *dst_scale,
              int accum, int sample, int32_t nsamp, int32_t ra, int32_t rb, float *Y,
              int64_t ldy) {
    const int32_t H = val ? val_heads : 1;
    const int32_t D = F / H;
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t r = 0; r < n_rows; ++r) {
        for (int32_t f = 0; f < F; ++f) {
            const int32_t h = f / D;
            const int start_from_y = accum && !dst_scale;
            float local = start_from_y ? Y[r * ldy + f] : 0.0f;
            for (int32_t s = 0; s < n_seg; ++s) {
                const int64_t e0 = SEG_BASE(s) + ROWPTR(s)[r];
                const int64_t e1 = SEG_BASE(s) + ROWPTR(s)[r + 1];
                const int32_t jmax = (int32_t)(e1 - e0);
                const int32_t nj = sample ? (jmax > 0 ? nsamp : 0) : jmax;
                for (int32_t ji = 0; ji < nj; ++ji) {
                    const int32_t j = sample ? (ra * ji + rb) % jmax : ji;
                    const int64_t e = e0 + j;
                    const int64_t c = col[e];
                    float v = X[c * ldx + f];
                    if (src_scale) v = src_scale[c] * v;
                    if (val)
                        local = fmaf(val[e * H + h], v, local);
                    else
                        local = local + v;
                }
            }
            if (dst_scale) {
                local = dst_scale[r] * local;
                if (accum) local = Y[r * ldy + f] + local;
            }
            Y[r * ldy + f] = local;
        }
    }
}

/* CPU baseline: the reference's gSpMM + wsumAgg restated (aggregators.h:12-31,55-127):
 * omp parallel for schedule(dynamic,1) over rows, accum[0:F] += w * X[u, 0:F] in CSR
 * order on the output row (caller zero-fills Y). */
void orc_gspmm(int64_t n_rows, const int32_t *rowptr, const int32_t *col, const float *val,
               const float *X, int32_t F, float *Y) {
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t v = 0; v < n_rows; ++v) {
        float *base1 = Y + v * (int64_t)F;
        for (int64_t e = rowptr[v]; e < rowptr[v + 1]; ++e) {
            const float w = val ? val[e] : 1.0f;
            const float *base2 = X + (int64_t)col[e] * F;
            for (int32_t j = 0; j < F; ++j) base1[j] = fmaf(w, base2[j], base1[j]);
        }
    }
}

/* Degree: aggregate_node_mul_sum_direct_*_call(ones, ...) (codegen/gala.cu:227-308,
 * 433-440) = sequential sum of A_e*1 (exact counts when unweighted), then
 * torch::pow(degrees, power).  Sampled graphs use FULL_OP n*S (common.h:1342-1374). */
void orc_degree(int64_t n_rows, int32_t n_seg, const int32_t *rowptr, const int32_t *seg_base,
                const float *val, float power, int sample, int32_t nsamp, float *deg) {
    for (int64_t r = 0; r < n_rows; ++r) {
        float d = 0.0f;
        if (sample) {
            d = (float)nsamp * (float)n_seg;
        } else {
            for (int32_t s = 0; s < n_seg; ++s)
                for (int64_t e = SEG_BASE(s) + ROWPTR(s)[r]; e < SEG_BASE(s) + ROWPTR(s)[r + 1]; ++e)
                    d = d + (val ? val[e] : 1.0f);
        }
        if (power != 1.0f) d = (power == -0.5f) ? 1.0f / sqrtf(d) : powf(d, power);
        deg[r] = d;
    }
}

/* SDDVV: default_function_kernel_sddvv_plus_undir (cuda.h:679-698): C[e] = A[row]+B[col_e];
 * default_function_kernel_sddvv_mult_undir (cuda.h:848-867): C[e] = A[row]*B[col_e];
 * op 2 appends torch::nn::LeakyReLU(slope) (common.h:1175-1184). heads: per-head columns. */
void orc_sddvv(int64_t n_rows, int32_t n_seg, const int32_t *rowptr, const int32_t *seg_base,
               const int32_t *col, const float *a, const float *b, int32_t H, int32_t op,
               float slope, float *out) {
    for (int32_t s = 0; s < n_seg; ++s)
        for (int64_t r = 0; r < n_rows; ++r)
            for (int64_t e = SEG_BASE(s) + ROWPTR(s)[r]; e < SEG_BASE(s) + ROWPTR(s)[r + 1]; ++e)
                for (int32_t h = 0; h < H; ++h) {
                    const float av = a[r * H + h], bv = b[(int64_t)col[e] * H + h];
                    float v = (op == 1) ? av * bv : av + bv;
                    if (op == 2) v = v > 0.0f ? v : v * slope;
                    out[e * H + h] = v;
                }
}

/* Edge->row sum: default_function_kernel_spmm_backward_sddmm_32_{nln,eaggr}
 * (cuda.h:505-524, 659-678): per segment launch local_C = 1e-12 (eps) then += A_e in
 * order; C[row] = C[row] + local_C.  Output zero-filled by the wrapper unless accum. */
void orc_row_sum(int64_t n_rows, int32_t n_seg, const int32_t *rowptr, const int32_t *seg_base,
                 const float *v, int32_t H, float eps, int accum, float *out) {
    for (int64_t r = 0; r < n_rows; ++r)
        for (int32_t h = 0; h < H; ++h) {
            float c = accum ? out[r * H + h] : 0.0f;
            for (int32_t s = 0; s < n_seg; ++s) {
                float local = eps;
                for (int64_t e = SEG_BASE(s) + ROWPTR(s)[r]; e < SEG_BASE(s) + ROWPTR(s)[r + 1]; ++e)
                    local = local + v[e * H + h];
                c = c + local;
            }
            out[r * H + h] = c;
        }
}

/* Row->edge scale: default_function_kernel_{softmax,mult}_sddvv_undir (cuda.h:525-562):
 * C[e] = C[e] * A[row], in place. */
void orc_row_scale(int64_t n_rows, int32_t n_seg, const int32_t *rowptr,
                   const int32_t *seg_base, const float *q, int32_t H, float *v) {
    for (int32_t s = 0; s < n_seg; ++s)
        for (int64_t r = 0; r < n_rows; ++r)
            for (int64_t e = SEG_BASE(s) + ROWPTR(s)[r]; e < SEG_BASE(s) + ROWPTR(s)[r + 1]; ++e)
                for (int32_t h = 0; h < H; ++h) v[e * H + h] = v[e * H + h] * q[r * H + h];
}

/* SDDMM dot: default_function_kernel_sddmm_mult_undir_shared (cuda.h:699-734) without
 * its shared-memory race: local_C = 0; for k: local_C = local_C + A[row,k]*B[col_e,k]
 * (fma); heads split the k range into H blocks of D. */
void orc_sddmm(int64_t n_rows, int32_t n_seg, const int32_t *rowptr, const int32_t *seg_base,
               const int32_t *col, const float *A, int64_t lda, const float *B, int64_t ldb,
               int32_t F, int32_t H, float *out) {
    const int32_t D = F / H;
    for (int32_t s = 0; s < n_seg; ++s)
        for (int64_t r = 0; r < n_rows; ++r)
            for (int64_t e = SEG_BASE(s) + ROWPTR(s)[r]; e < SEG_BASE(s) + ROWPTR(s)[r + 1]; ++e)
                for (int32_t h = 0; h < H; ++h) {
                    float local = 0.0f;
                    for (int32_t k = h * D; k < (h + 1) * D; ++k)
                        local = fmaf(A[r * lda + k], B[(int64_t)col[e] * ldb + k], local);
                    out[e * H + h] = local;
                }
}

/* Edge softmax forward, REF mode = non_lnr_op_softmax_AutoGrad::forward
 * (common.h:760-773): val_exp = clamp(exp(s), 0, 1e12); row_sum = K7(val_exp) (eps
 * 1e-12 per segment); row_sum = reciprocal(row_sum); alpha = K8(row_sum, val_exp).
 * FIXED mode: alpha = exp(s - max_row) / sum_row exp(s - max_row). */
void orc_softmax_fwd(int64_t n_rows, int32_t n_seg, const int32_t *rowptr,
                     const int32_t *seg_base, const float *logit, int32_t H, int mode,
                     float *alpha) {
    for (int64_t r = 0; r < n_rows; ++r)
        for (int32_t h = 0; h < H; ++h) {
            if (mode == 0) {
                float c = 0.0f;
                for (int32_t s = 0; s < n_seg; ++s) {
                    float local = 1e-12f;
                    for (int64_t e = SEG_BASE(s) + ROWPTR(s)[r]; e < SEG_BASE(s) + ROWPTR(s)[r + 1]; ++e) {
                        float p = expf(logit[e * H + h]);
                        p = p > 1e12f ? 1e12f : p;
                        local = local + p;
                    }
                    c = c + local;
                }
                const float q = 1.0f / c;
                for (int32_t s = 0; s < n_seg; ++s)
                    for (int64_t e = SEG_BASE(s) + ROWPTR(s)[r]; e < SEG_BASE(s) + ROWPTR(s)[r + 1]; ++e) {
                        float p = expf(logit[e * H + h]);
                        p = p > 1e12f ? 1e12f : p;
                        alpha[e * H + h] = p * q;
                    }
            } else {
                float m = -INFINITY;
                for (int32_t s = 0; s < n_seg; ++s)
                    for (int64_t e = SEG_BASE(s) + ROWPTR(s)[r]; e < SEG_BASE(s) + ROWPTR(s)[r + 1]; ++e)
                        m = fmaxf(m, logit[e * H + h]);
                double sum = 0.0;
                for (int32_t s = 0; s < n_seg; ++s)
                    for (int64_t e = SEG_BASE(s) + ROWPTR(s)[r]; e < SEG_BASE(s) + ROWPTR(s)[r + 1]; ++e)
                        sum += exp((double)logit[e * H + h] - m);
                for (int32_t s = 0; s < n_seg; ++s)
                    for (int64_t e = SEG_BASE(s) + ROWPTR(s)[r]; e < SEG_BASE(s) + ROWPTR(s)[r + 1]; ++e)
                        alpha[e * H + h] = (float)(exp((double)logit[e * H + h] - m) / sum);
            }
        }
}

/* Edge softmax backward = non_lnr_op_softmax_AutoGrad::backward (common.h:791-799):
 * sds = alpha*d_alpha; accum = K7(sds) (eps per segment, REF only);
 * res = K8(accum, alpha); d_logit = sds - res. */
void orc_softmax_bwd(int64_t n_rows, int32_t n_seg, const int32_t *rowptr,
                     const int32_t *seg_base, const float *alpha, const float *dalpha,
                     int32_t H, int mode, float *dlogit) {
    const float eps = mode == 0 ? 1e-12f : 0.0f;
    for (int64_t r = 0; r < n_rows; ++r)
        for (int32_t h = 0; h < H; ++h) {
            float c = 0.0f;
            for (int32_t s = 0; s < n_seg; ++s) {
                float local = eps;
                for (int64_t e = SEG_BASE(s) + ROWPTR(s)[r]; e < SEG_BASE(s) + ROWPTR(s)[r + 1]; ++e)
                    local = local + alpha[e * H + h] * dalpha[e * H + h];
                c = c + local;
            }
            for (int32_t s = 0; s < n_seg; ++s)
                for (int64_t e = SEG_BASE(s) + ROWPTR(s)[r]; e < SEG_BASE(s) + ROWPTR(s)[r + 1]; ++e) {
                    const float sds = alpha[e * H + h] * dalpha[e * H + h];
                    dlogit[e * H + h] = sds - alpha[e * H + h] * c;
                }
        }
}

/* ---- CPU baseline of the SDDMM + edge-softmax half ------------------------------------
 * One REF GAT layer (single segment CSR, H heads of D features), forward + backward, pass
 * by pass exactly as the generated program composes it, every pass an
 * OpenMP loop over the rows [0, n_rows).  Each pass is the restatement of one reference
 * kernel or torch op, with the rounding of the single-pass functions above, so the result
 * is bit-identical to composing orc_sddvv / orc_softmax_fwd / orc_spmm / orc_sddmm /
 * orc_softmax_bwd / orc_row_sum (tests/test_cpu_baseline.py):
 *   forward   aR[r] = <X[r, head h], wR_h> + bR_h   attnR = efc(res), per head (common.h:1248-1260)
 *             s = aL[r] + aR[c]                    K5 sddvv_plus   (cuda.h:679-698)
 *             t = LeakyReLU(s)                     torch           (common.h:1175-1184)
 *             p = clamp(exp(t), 0, 1e12)           torch exp, clamp (common.h:760-766)
 *             rs = 1e-12 + sum_row p; q = 1/rs     K7 + reciprocal (cuda.h:505-524; common.h:767-770)
 *             alpha = p * q                        K8 in place     (cuda.h:525-562)
 *             Y[r] = sum alpha_e X[c]              K1 weighted     (cuda.h:286-358)
 *   backward  dX[r] = sum alpha_e dY[c]            SpMM on slot 2li+1, forward alpha (common.h:835-894)
 *             da_e = <dY[r], X[c]>                 K9 sddmm        (cuda.h:699-734)
 *             sds = alpha*da; acc = 1e-12 + sum_row sds; res = acc*alpha; ds = sds - res
 *                                                  softmax bwd     (common.h:791-799)
 *             dt = where(s > 0, ds, ds*slope)      LeakyReLU bwd
 *             daL[r] = 1e-12 + sum_row dt          K7              (cuda.h:505-524)
 * aR must hold the rows >= n_rows already (orc_head_attn); the layer recomputes rows
 * [0, n_rows) itself, so a row sample does a proportional share of that pass.  Edge
 * buffers s, pa (t -> p -> alpha), da (da -> sds -> ds -> dt), res: [nnz(n_rows), H]. */
void orc_head_attn(int64_t r0, int64_t r1, const float *X, int64_t ldx, int32_t H, int32_t D,
                   const float *wR, const float *bR, float *aR) {
#pragma omp parallel for schedule(static)
    for (int64_t r = r0; r < r1; ++r)
        for (int32_t h = 0; h < H; ++h) {
            float acc = 0.0f;
            for (int32_t k = 0; k < D; ++k) acc = fmaf(X[r * ldx + h * D + k], wR[h * D + k], acc);
            aR[r * H + h] = acc + (bR ? bR[h] : 0.0f);
        }
}

#define ROWS_OMP _Pragma("omp parallel for schedule(dynamic, 256)") for (int64_t r = 0; r < n_rows; ++r)
#define EDGES for (int64_t e = rowptr[r]; e < rowptr[r + 1]; ++e)

/* rid (nullable): row r of the CSR given is the layer's row rid[r] (a row sample of a larger
 * graph: aL and the row side of dY are read at rid[r], columns stay global, outputs at r);
 * aR must then hold every row already (no recompute). */
static void gat_ref_layer(int64_t n_rows, const int32_t *rowptr, const int32_t *col, int32_t H,
                          int32_t D, const float *aL, const float *X, const float *wR,
                          const float *bR, const float *dY, float slope, float *aR, float *s,
                          float *pa, float *da, float *res, float *q, float *Y, float *dX,
                          float *daL, const int64_t *rid) {
    const int32_t F = H * D;
    if (!rid) orc_head_attn(0, n_rows, X, F, H, D, wR, bR, aR);
#define RID (rid ? rid[r] : r)
    ROWS_OMP EDGES for (int32_t h = 0; h < H; ++h) s[e * H + h] = aL[RID * H + h] + aR[(int64_t)col[e] * H + h];
    ROWS_OMP EDGES for (int32_t h = 0; h < H; ++h) {
        const float v = s[e * H + h];
        pa[e * H + h] = v > 0.0f ? v : v * slope;
    }
    ROWS_OMP EDGES for (int32_t h = 0; h < H; ++h) pa[e * H + h] = expf(pa[e * H + h]);
    ROWS_OMP EDGES for (int32_t h = 0; h < H; ++h) pa[e * H + h] = pa[e * H + h] > 1e12f ? 1e12f : pa[e * H + h];
    ROWS_OMP for (int32_t h = 0; h < H; ++h) {
        float local = 1e-12f;
        EDGES local = local + pa[e * H + h];
        q[r * H + h] = 0.0f + local;
    }
    ROWS_OMP for (int32_t h = 0; h < H; ++h) q[r * H + h] = 1.0f / q[r * H + h];
    ROWS_OMP EDGES for (int32_t h = 0; h < H; ++h) pa[e * H + h] = pa[e * H + h] * q[r * H + h];
    ROWS_OMP for (int32_t f = 0; f < F; ++f) {
        float local = 0.0f;
        EDGES local = fmaf(pa[e * H + f / D], X[(int64_t)col[e] * F + f], local);
        Y[r * F + f] = local;
    }
    /* backward */
    ROWS_OMP for (int32_t f = 0; f < F; ++f) {
        float local = 0.0f;
        EDGES local = fmaf(pa[e * H + f / D], dY[(int64_t)col[e] * F + f], local);
        dX[r * F + f] = local;
    }
    ROWS_OMP EDGES for (int32_t h = 0; h < H; ++h) {
        float local = 0.0f;
        for (int32_t k = h * D; k < (h + 1) * D; ++k)
            local = fmaf(dY[RID * F + k], X[(int64_t)col[e] * F + k], local);
        da[e * H + h] = local;
    }
    ROWS_OMP EDGES for (int32_t h = 0; h < H; ++h) da[e * H + h] = pa[e * H + h] * da[e * H + h];
    ROWS_OMP for (int32_t h = 0; h < H; ++h) {
        float local = 1e-12f;
        EDGES local = local + da[e * H + h];
        daL[r * H + h] = 0.0f + local;             /* acc, parked in daL until the last pass */
    }
    ROWS_OMP EDGES for (int32_t h = 0; h < H; ++h) res[e * H + h] = pa[e * H + h] * daL[r * H + h];
    ROWS_OMP EDGES for (int32_t h = 0; h < H; ++h) da[e * H + h] = da[e * H + h] - res[e * H + h];
    ROWS_OMP EDGES for (int32_t h = 0; h < H; ++h) {
        const float d = da[e * H + h];
        da[e * H + h] = s[e * H + h] > 0.0f ? d : d * slope;
    }
    ROWS_OMP for (int32_t h = 0; h < H; ++h) {
        float local = 1e-12f;
        EDGES local = local + da[e * H + h];
        daL[r * H + h] = 0.0f + local;
    }
#undef RID
}

void orc_gat_ref_layer(int64_t n_rows, const int32_t *rowptr, const int32_t *col, int32_t H,
                       int32_t D, const float *aL, const float *X, const float *wR,
                       const float *bR, const float *dY, float slope, float *aR, float *s,
                       float *pa, float *da, float *res, float *q, float *Y, float *dX,
                       float *daL) {
    gat_ref_layer(n_rows, rowptr, col, H, D, aL, X, wR, bR, dY, slope, aR, s, pa, da, res, q, Y, dX,
                  daL, NULL);
}

void orc_gat_ref_layer_rows(int64_t n_rows, const int32_t *rowptr, const int32_t *col, int32_t H,
                            int32_t D, const float *aL, const float *X, const float *wR,
                            const float *bR, const float *dY, float slope, float *aR, float *s,
                            float *pa, float *da, float *res, float *q, float *Y, float *dX,
                            float *daL, const int64_t *rid) {
    gat_ref_layer(n_rows, rowptr, col, H, D, aL, X, wR, bR, dY, slope, aR, s, pa, da, res, q, Y, dX,
                  daL, rid);
}
#undef ROWS_OMP
#undef EDGES

/* OpenMP team size for the CPU-baseline loops (bench.py: every core the process may use) */
void orc_set_threads(int n) { omp_set_num_threads(n); }

/* ---- graph layout -------------------------------------------------------------------- */

/* CSRCMatrix::build (csrc_matrix.h:148-376) as called by readSM_npy32 (tests/common.h:
 * 331-366): counting sort by row (count_atomic + partial_sum + count_sort_place_2arr,
 * mtx_sort.h:52-137,165-174), then each row's columns sorted ascending (sort_range2arr,
 * mtx_sort.h:683-722); duplicates kept.  Sequential stable restatement. */
int orc_csr_build(int64_t n_rows, int64_t nnz, const int32_t *src, const int32_t *dst,
                  int32_t *rowptr, int32_t *col) {
    int64_t *cnt = (int64_t *)calloc((size_t)n_rows + 1, sizeof(int64_t));
    if (!cnt) return -1;
    for (int64_t e = 0; e < nnz; ++e) cnt[src[e] + 1]++;
    for (int64_t r = 0; r < n_rows; ++r) cnt[r + 1] += cnt[r];
    for (int64_t r = 0; r <= n_rows; ++r) rowptr[r] = (int32_t)cnt[r];
    for (int64_t e = 0; e < nnz; ++e) col[cnt[src[e]]++] = dst[e];
    for (int64_t r = 0; r < n_rows; ++r) { /* insertion sort: rows are short in fixtures */
        for (int64_t i = rowptr[r] + 1; i < rowptr[r + 1]; ++i) {
            const int32_t x = col[i];
            int64_t j = i - 1;
            while (j >= rowptr[r] && col[j] > x) {
                col[j + 1] = col[j];
                --j;
            }
            col[j + 1] = x;
        }
    }
    free(cnt);
    return 0;
}

/* static_ord_col_breakpoints (tiling.h:1594-1608) + ord_col_tiling_torch
 * (tiling.h:222-283): segment s keeps, row by row, the edges with col in [j_s, j_{s+1});
 * offsets are relative to the segment's first edge, bounds = [start, end).  Returns S. */
int32_t orc_col_tile(int64_t n_rows, int64_t n_cols, const int32_t *rowptr, const int32_t *col,
                     const float *val, int32_t cols_per_partition, int32_t *out_rowptr,
                     int32_t *out_col, float *out_val, int32_t *out_bounds) {
    int32_t nseg = 0;
    int64_t new_nvals = 0, prev_nvals = 0;
    for (int64_t j0 = 0; j0 < n_cols; j0 += cols_per_partition, ++nseg) {
        const int64_t j1 = (j0 + cols_per_partition < n_cols) ? j0 + cols_per_partition : n_cols;
        int32_t *orp = out_rowptr + (int64_t)nseg * (n_rows + 1);
        orp[0] = (int32_t)(new_nvals - prev_nvals);
        out_bounds[2 * nseg] = (int32_t)new_nvals;
        for (int64_t r = 0; r < n_rows; ++r) {
            for (int64_t e = rowptr[r]; e < rowptr[r + 1]; ++e) {
                if (col[e] >= j0 && col[e] < j1) {
                    out_col[new_nvals] = col[e];
                    if (out_val) out_val[new_nvals] = val ? val[e] : 1.0f;
                    new_nvals++;
                }
            }
            orp[r + 1] = (int32_t)(new_nvals - prev_nvals);
        }
        out_bounds[2 * nseg + 1] = (int32_t)new_nvals;
        prev_nvals = new_nvals;
    }
    return nseg;
}

static int cmp_i32(const void *a, const void *b) {
    const int32_t x = *(const int32_t *)a, y = *(const int32_t *)b;
    return (x > y) - (x < y);
}

/* inplace_sample_graph_ab (tiling.h:454-508): per row, e_used = {first + (ra*ji+rb) %
 * total_e : ji < n}, sorted; new offsets i*n. */
int orc_sample_ab(int64_t n_rows, const int32_t *rowptr, const int32_t *col, const float *val,
                  int32_t nsamp, int32_t ra, int32_t rb, int32_t *out_rowptr, int32_t *out_col,
                  float *out_val) {
    int32_t *used = (int32_t *)malloc(sizeof(int32_t) * (nsamp > 0 ? nsamp : 1));
    out_rowptr[0] = 0;
    for (int64_t i = 0; i < n_rows; ++i) {
        const int32_t first = rowptr[i], total = rowptr[i + 1] - rowptr[i];
        if (total == 0 && nsamp > 0) {
            free(used);
            return -1;
        }
        for (int32_t ji = 0; ji < nsamp; ++ji) used[ji] = first + (ra * ji + rb) % total;
        qsort(used, (size_t)nsamp, sizeof(int32_t), cmp_i32);
        for (int32_t j = 0; j < nsamp; ++j) {
            out_col[i * nsamp + j] = col[used[j]];
            if (out_val) out_val[i * nsamp + j] = val ? val[used[j]] : 1.0f;
        }
        out_rowptr[i + 1] = (int32_t)((i + 1) * nsamp);
    }
    free(used);
    return 0;
}

/* getMaskSubgraphs, one level (tests/common.h:21-110): rows with mask > 0 keep all
 * their edges in order, the others become empty; next[i] = max(0, max_{e in row i}
 * mask[col_e]) (gSpMM with maxAgg into a zero-initialised vector, :103-107). */
int orc_mask_subgraph(int64_t n_rows, const int32_t *rowptr, const int32_t *col,
                      const int32_t *mask, int32_t *out_rowptr, int32_t *out_col,
                      int32_t *next) {
    int64_t k = 0;
    out_rowptr[0] = 0;
    for (int64_t i = 0; i < n_rows; ++i) {
        if (mask[i] > 0)
            for (int32_t e = rowptr[i]; e < rowptr[i + 1]; ++e) out_col[k++] = col[e];
        out_rowptr[i + 1] = (int32_t)k;
    }
    for (int64_t i = 0; i < n_rows; ++i) {
        int32_t m = 0;
        for (int32_t e = rowptr[i]; e < rowptr[i + 1]; ++e)
            if (mask[col[e]] > m) m = mask[col[e]];
        next[i] = m;
    }
    return 0;
}
