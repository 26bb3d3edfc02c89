/*
 * gala_hip.h — C ABI of libgala_hip.so, the MI355X (gfx950) hot path of GALA's
 * generated GNN programs: SpMM neighbour aggregation, SDDVV/SDDMM, edge-softmax and
 * the per-edge / per-row scalings around them, plus the host-side graph-layout
 * builders those kernels consume.
 *
 * Every entry point replaces one free function that GALA's CUDA code generator emits
 * into gala.cu (src/codegen/cuda.h) or one host routine that gala.cu includes
 * textually (src/formats, src/ops).  The reference interface each one replaces is
 * cited as path:line relative to the GALA repository root.
 *
 * Conventions (all entry points):
 *   - Plain C types only.  No torch/HIP types in the signatures; `stream` is a
 *     hipStream_t passed as void* (NULL = the legacy null stream).
 *   - Device pointers unless a parameter is documented HOST.  All memory is owned by
 *     the caller; the library never allocates device memory and never synchronises
 *     the device, so every call is capturable into a hipGraph.
 *   - Return 0 (GALA_OK) or a negative gala_status.  The library never exits
 *     (the reference prints and exit()s from CUDA_CHECK, codegen/gala.cu:46-64).
 *   - Reentrant: no process globals except a thread-local last-HIP-error code.
 *   - Indices are int32 (as in the reference, cuda.h:286-358); all address
 *     arithmetic inside the kernels is 64-bit, so N*F >= 2^31 is supported
 *     (the reference's `row*dcols` overflows there, SURVEY §7 hard part 3).
 */
#ifndef GALA_HIP_H
#define GALA_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GALA_ABI_VERSION 6

typedef enum gala_status {
    GALA_OK = 0,
    GALA_ERR_INVALID_ARG = -1, /* null pointer, negative size, bad flag/mode, misaligned ld  */
    GALA_ERR_UNSUPPORTED = -2, /* shape the library does not implement (reported, not UB)    */
    GALA_ERR_HIP = -3,         /* a HIP runtime call failed; see gala_last_hip_error()         */
    GALA_ERR_GRAPH = -4        /* malformed graph (rowptr not monotone, col out of range, ...) */
} gala_status;

/* ------------------------------------------------------------------------------------
 * Graph descriptor.
 *
 * Mirrors the device-side graph the generated code keeps in the global slots
 * global_offset_graph / global_columns_graph / global_value_graph / global_bounds /
 * global_segments (codegen/gala.cu:32-43, emitted by src/codegen/common.h:1694-1705).
 *
 * n_seg == 1: plain CSR, rowptr[n_rows+1], rows sorted, cols ascending inside a row,
 *             duplicates kept (CSRCMatrix::build, src/formats/csrc_matrix.h:148-376).
 * n_seg  > 1: the column-tiled layout produced by ord_col_tiling_torch
 *             (src/ops/tiling.h:222-283): rowptr holds n_seg blocks of n_rows+1
 *             RELATIVE offsets, segment s's edges start at col[seg_bounds[2s]].
 *             Aggregation over a tiled graph is defined as the ordered sum over the
 *             segments (the reference launches segments on racing streams,
 *             cuda.h:472-499; here segment 0 is accumulated first, then 1, ...).
 * ---------------------------------------------------------------------------------- */
/*
 * Optional split plan for power-law graphs, built once per graph on the host with
 * gala_host_split_plan (only used for n_seg == 1).  Rows longer than `threshold` edges are
 * hub rows.  By default (REF order, the reference's serial row loop, cuda.h:286-358) the
 * SpMM sums a hub row sequentially in CSR order like every other row -- bit-identical to
 * the reference -- in a dedicated kernel whose workgroup gathers a tile of the row's
 * neighbour rows while one wave runs the row's add chain (k_spmm_hub_exact); with
 * `aux_stream` and `aux_events` set it runs on that stream beside the row kernel (an
 * event fork / join on the caller's stream: stream-ordered, hipGraph-capturable).  With
 * GALA_SPMM_HUB_CHUNKED (the fast, reordered mode) a hub row is instead cut into chunks of
 * `chunk` edges that run in parallel; each chunk writes a partial sum to `workspace` and a
 * fix-up pass adds the partials of a row in chunk order, so those rows match the reference
 * within fp32 summation rounding instead of bit for bit.  gala_row_sum_f32 sums hub rows the
 * same two ways; the softmax and GAT kernels always use the chunks (their row sums are
 * reductions the GPU regroups anyway, measured within 1e-4 on 388 K-edge rows).
 */
typedef struct gala_split_plan {
    int32_t threshold;         /* rows with deg > threshold are hub rows                 */
    int32_t chunk;             /* edges per chunk                                        */
    int64_t n_rows_split;
    int64_t n_chunks;
    const int32_t *rows;       /* device [n_rows_split]: hub row ids (ascending)         */
    const int32_t *row_chunk0; /* device [n_rows_split+1]: first chunk of each split row  */
    const int32_t *chunk_row;  /* device [n_chunks]: index into rows[] of every chunk    */
    float *workspace;          /* device [n_chunks * ws_cols] partial results            */
    int64_t ws_cols;           /* floats per chunk (>= F for SpMM, >= F + 2*heads GAT)    */
    const int32_t *row_order;  /* device [n_rows] or NULL: the SpMM processes rows in this
                                  order (gala_host_row_order: by descending degree), so the
                                  rows sharing a wavefront have similar lengths on skewed
                                  graphs; results are unchanged (every row is still one
                                  sequential pass).  A plan may carry only a row order
                                  (n_chunks == 0).  With hub rows it must be that order
                                  of the same rowptr: its first n_rows_split entries are
                                  then the hub rows, longest first, the order in which
                                  the REF-order hub kernel takes them.                   */
    void *aux_stream;          /* hipStream_t or NULL: where the REF-order hub rows run   */
    void *aux_events[2];       /* hipEvent_t fork / join pair for aux_stream (both or none).
                                  Every hub fork of the plan (gala_spmm_ex_f32,
                                  gala_row_sum_f32) records and waits on these two events,
                                  so a plan serves ONE caller stream at a time: calls on one
                                  graph from two host threads / streams must be ordered by
                                  the caller (or use a plan each), else one call's join can
                                  wait on the other's fork.                               */
} gala_split_plan_t;

typedef struct gala_csr {
    int64_t n_rows;            /* rows of A (destination vertices of the aggregation)     */
    int64_t n_cols;            /* columns of A (source vertices); X has n_cols rows      */
    int64_t nnz;               /* stored edges over all segments                          */
    const int32_t *rowptr;     /* device [(n_rows+1)*n_seg]                               */
    const int32_t *col;        /* device [nnz]                                            */
    const float *val;          /* device [nnz*val_heads] or NULL = unweighted (A_e = 1)   */
    int32_t val_heads;         /* edge values per edge (1 = reference; H for multi-head) */
    int32_t n_seg;             /* >= 1                                                    */
    const int32_t *seg_bounds; /* HOST [2*n_seg] {start,end} edge of each segment, or
                                  NULL when n_seg == 1 (reference keeps `bounds` on the
                                  host: cuda.h:472-475 reads bounds_ptr on the CPU)        */
    const gala_split_plan_t *split; /* HOST pointer, NULL = no row splitting              */
    const float *val_row_scale; /* device [n_rows*val_heads] or NULL: the edge values are
                                   stored factored, A_e,h = val[e,h] * val_row_scale[row,h]
                                   (rounded product).  The GAT forward's factored attention
                                   output (gala_gat_fwd_ex_f32: p and q) is used this way as
                                   the backward's alpha without materialising it.  Only the
                                   SpMM and the GAT backward read it.                      */
} gala_csr_t;

/* ---- library information ------------------------------------------------------------ */
int gala_abi_version(void);
const char *gala_status_string(int status);
int gala_last_hip_error(void);                 /* hipError_t of the last GALA_ERR_HIP    */

/* ---- SpMM neighbour aggregation ----------------------------------------------------- */
#define GALA_SPMM_ACCUM 0x1   /* Y += result (reference: wrapper zero-fills Y, kernel adds,
                                 cuda.h:463 + 309-310); without it Y is overwritten       */
#define GALA_SPMM_SAMPLE 0x2  /* kernel sampling: per row with deg>0, nsamp edges
                                 j = (ra*ji + rb) mod deg (cuda.h:313-321)                */
#define GALA_SPMM_EXACT 0x4   /* every row in one sequential pass (the default since ABI 3;
                                 kept as an explicit request; excludes HUB_CHUNKED)       */
#define GALA_SPMM_HUB_CHUNKED 0x8 /* hub rows of A->split as chunk partials + ordered fix-up:
                                 the fast mode, within fp32 summation rounding of REF     */

/*
 * Y[r, 0:F] (+)= dst_scale[r] * sum_{e in row r} w_e * (src_scale[col_e] * X[col_e, 0:F])
 *
 * w_e = val[e*val_heads + h] for the head h = f / (F/val_heads) of feature f
 * (= 1 when val == NULL).  src_scale/dst_scale may be NULL (= 1); they fuse the GCN
 * `norm * res` row broadcasts the generated forward wraps around every aggregation
 * (codegen/gala.cu:442-456) with the reference's rounding (product rounded before
 * the sum).  Edges are accumulated sequentially in CSR order per row, in fp32, with
 * the same fma contraction nvcc applies to the emitted kernel, so results are
 * bit-identical to the reference kernel for every input.
 *
 * Replaces: <aggregate_node_mul_sum[_direct]_coarse{C}>_call (cuda.h:441-502,
 *           emitted codegen/gala.cu:227-390) and its kernels _kernel{k}/_offset
 *           (cuda.h:286-436), the cuSPARSE "gather_forward" path (cuda.h:211-279),
 *           and the kernel-sampled variants (cuda.h:313-321,389-397).
 * ldx/ldy are row strides in elements (>= F).
 */
int gala_spmm_f32(const gala_csr_t *A, const float *X, int64_t ldx, float *Y, int64_t ldy,
                  int32_t F, const float *src_scale, const float *dst_scale, int32_t flags,
                  int32_t nsamp, int32_t ra, int32_t rb, void *stream);

/*
 * gala_spmm_ex_f32: gala_spmm_f32 with an epilogue (NULL: none), for the GCN step
 * `norm * A (norm * H)` of codegen/gala.cu:433-456 without the separate degree and
 * ROW_BROADCAST passes:
 *   dst_deg_rsqrt = 1: the dst factor of row r is deg(r)^-0.5 computed from A's rowptr --
 *                   the exact values gala_degree_f32(power -0.5) gives on an unweighted
 *                   graph (dst_scale must be NULL; one segment; A->val NULL -- a weighted
 *                   graph's degree sums its values: GALA_ERR_UNSUPPORTED; not with
 *                   GALA_SPMM_SAMPLE);
 *   Y2 != NULL:     also Y2[r, 0:F] = s2[r] * Y[r, 0:F] (s2 = y2_scale, or the dst factor
 *                   when NULL), rounded as the ROW_BROADCAST the next aggregation's input
 *                   would be -- bit-identical to that pass over Y.
 */
typedef struct gala_spmm_epilogue {
    int32_t dst_deg_rsqrt;
    float *Y2;
    int64_t ldy2;
    const float *y2_scale;
    /* ABI 4: the ReLU of a GCN layer on either side of the aggregation (gala_torch's
     * gcn_aggregate_relu_apply), each element with the roundings of the separate pass:
     *   src_relu = 1:   the gathered source is src_scale[c] * relu(src_act[c] * X[c]) -- the
     *                   next layer's prologue, gala_row_scale_relu_f32(act = src_act, pre =
     *                   src_scale) -- src_act / src_scale may be NULL (factor 1);
     *   relu_x != NULL: the ReLU backward of the layer's input, applied to the result:
     *                   Y[r] = relu_act[r] * (relu(relu_act[r] * relu_x[r]) <= 0 ? 0 : Y[r])
     *                   (gala_relu_scale_backward_f32; relu_act may be NULL), relu_x [n_rows,
     *                   ldrx >= F] row-major.
     * Both: unweighted, unsampled, without a hub-row plan (A->split with hub rows) and without
     * Y2; else GALA_ERR_UNSUPPORTED.  (relu: t > 0 ? t : +0, NaN passes -- torch.relu on the
     * GPU.) */
    int32_t src_relu;
    const float *src_act;
    const float *relu_x;
    int64_t ldrx;
    const float *relu_act;
} gala_spmm_epilogue_t;
int gala_spmm_ex_f32(const gala_csr_t *A, const float *X, int64_t ldx, float *Y, int64_t ldy, int32_t F,
                     const float *src_scale, const float *dst_scale, int32_t flags, int32_t nsamp,
                     int32_t ra, int32_t rb, const gala_spmm_epilogue_t *epi, void *stream);
/* Y[r, :] = deg(r)^-0.5 * X[r, :] with deg from A's rowptr (one segment, unweighted: A->val
 * set gives GALA_ERR_UNSUPPORTED): the degree pass, pow(-0.5) and the `norm * X`
 * ROW_BROADCAST in one elementwise pass, bit-identical to them. */
int gala_row_broadcast_deg_f32(const gala_csr_t *A, int32_t F, const float *X, int64_t ldx, float *Y,
                               int64_t ldy, void *stream);

/*
 * deg[r] = sum_{e in row r} (val ? val[e] : 1)  (exact integer counts for unweighted
 * graphs), then deg[r] = deg[r]^power when power != 1 (fuses torch::pow(degrees,-0.5),
 * codegen/gala.cu:437-440).  With GALA_SPMM_SAMPLE the degree of the kernel-sampled
 * graph is used: nsamp * n_seg for every row, as FULL_OP does (common.h:1342-1374).
 * Replaces: aggregate_node_mul_sum_direct_coarse{C}_call(ones, ...) (codegen/gala.cu:227-308).
 */
int gala_degree_f32(const gala_csr_t *A, float *deg, float power, int32_t flags, int32_t nsamp,
                    void *stream);

/*
 * Y[r, 0:F] = scale[r] * X[r, 0:F]  (rounded product, torch `norm * res`).
 * Replaces: the ROW_BROADCAST_OP the generated forward applies around every GCN
 * aggregation (src/codegen/common.h:1150-1169, emitted codegen/gala.cu:442-456).
 * Y may alias X (in place) when ldy == ldx.
 */
int gala_row_broadcast_f32(int64_t n_rows, int32_t F, const float *scale, const float *X,
                           int64_t ldx, float *Y, int64_t ldy, void *stream);

/*
 * Y[r, 0:F] = pre[r] * relu(act[r] * X[r, 0:F]), relu(t) = t > 0 ? t : +0 with NaN passing
 * through (torch.relu's GPU kernel); act and/or pre may be NULL (no factor, no rounding step).
 * Replaces: the elementwise chain the generated forward runs in front of a GCN
 * aggregation -- ROW_BROADCAST (`norm * res`, common.h:1150-1169), NON_LNR_OP_RELU
 * (common.h:1170-1174), and the next layer's ROW_BROADCAST -- as one pass, with the same
 * roundings (bit-identical to the three torch ops).
 */
int gala_row_scale_relu_f32(int64_t n_rows, int32_t F, const float *act, const float *pre,
                            const float *X, int64_t ldx, float *Y, int64_t ldy, void *stream);

/*
 * Backward of the ReLU prologue: dX[r, :] = act[r] * (act[r] * X[r, :] <= 0 ? 0 : G[r, :])
 * (torch's threshold_backward on the ReLU output, then the product rule of act * X; act
 * may be NULL).  G is the gradient of relu(act * X).
 */
int gala_relu_scale_backward_f32(int64_t n_rows, int32_t F, const float *act, const float *X,
                                 int64_t ldx, const float *G, int64_t ldg, float *dX,
                                 int64_t lddx, void *stream);

/* ---- edge (SDDVV / SDDMM) ops -------------------------------------------------------- */
#define GALA_SDDVV_ADD 0        /* out[e,h] = a[row,h] + b[col_e,h]   (cuda.h:679-698)     */
#define GALA_SDDVV_MUL 1        /* out[e,h] = a[row,h] * b[col_e,h]   (cuda.h:848-867)     */
#define GALA_SDDVV_ADD_LRELU 2  /* ADD followed by LeakyReLU(slope) (common.h:1175-1184)   */

/*
 * Replaces: edge_sddvv (cuda.h:773-807), aggregate_edge_mul / aggregate_edge_mul_dir
 *           (cuda.h:870-952).  a_row/b_col are [n_rows,heads] / [n_cols,heads].
 */
int gala_sddvv_f32(const gala_csr_t *A, const float *a_row, const float *b_col, int32_t heads,
                   int32_t op, float slope, float *out_e, void *stream);

/*
 * out[r,h] (+)= sum_s ( eps + sum_{e in row r, segment s} v[e,h] )
 * in the reference's order: per segment local = eps, then local + v[e,h] for the segment's
 * edges in CSR order, added to the row's value (segment 0 first) -- bit-identical, hub rows of
 * A->split included (summed by one serial chain each, on the plan's side stream when it has
 * one).
 * Replaces: node_spmv_backward_of_sddmm_{nln,eaggr} (cuda.h:565-600, 737-772; kernels
 *           505-524, 659-678 start each segment's per-row sum at 1e-12).
 * flags: GALA_SPMM_ACCUM adds into out_row, otherwise out_row is overwritten;
 *        GALA_SPMM_HUB_CHUNKED sums the hub rows as chunk partials + an ordered fix-up (the
 *        fast mode, within fp32 summation rounding; needs the plan's workspace, 2 * heads
 *        floats per chunk).
 */
int gala_row_sum_f32(const gala_csr_t *A, const float *v_e, int32_t heads, float eps,
                     float *out_row, int32_t flags, void *stream);

/*
 * v[e,h] *= q[row,h] in place.
 * Replaces: inplace_softmax_sddvv / inplace_softmax_sddvv_mult (cuda.h:601-656,
 *           kernels 525-562).
 */
int gala_row_scale_f32(const gala_csr_t *A, const float *q_row, int32_t heads, float *v_inout,
                       void *stream);

/*
 * out[e,h] = sum_{k in head h} Ad[row,k] * Bd[col_e,k]   (F = heads*D features)
 * Replaces: edge_sddmm (cuda.h:808-845, kernel 699-734; the reference stages Ad's row in
 *           a block-shared LDS buffer that all 8 rows of a block overwrite — a race,
 *           SURVEY §5 — here every row owns its slab).
 */
int gala_sddmm_dot_f32(const gala_csr_t *A, const float *Ad, int64_t lda, const float *Bd,
                       int64_t ldb, int32_t F, int32_t heads, float *out_e, void *stream);

/* ---- edge softmax ------------------------------------------------------------------- */
#define GALA_SOFTMAX_REF 0    /* reference: p=min(exp(s),1e12), alpha = p*(1/(S*1e-12+sum p)),
                                 no max subtraction (common.h:760-773)                    */
#define GALA_SOFTMAX_FIXED 1  /* numerically stable: alpha = exp(s-max)/sum exp(s-max)    */

/*
 * alpha[e,h] = softmax over the edges of row(e) of logits[.,h].
 * Replaces: non_lnr_op_softmax_AutoGrad::forward (common.h:760-773: torch::exp,
 *           torch::clamp, K7 row-sum, torch::reciprocal, K8 row-scale).
 */
int gala_edge_softmax_fwd_f32(const gala_csr_t *A, const float *logits, int32_t heads,
                              int32_t mode, float *alpha, void *stream);

/*
 * d_logits[e] = alpha[e]*d_alpha[e] - alpha[e]*(S*eps + sum_{row} alpha*d_alpha)
 * (eps = 1e-12 in REF mode, 0 in FIXED mode).
 * Replaces: non_lnr_op_softmax_AutoGrad::backward (common.h:791-799), without the
 *           reference's in-place overwrite of the saved alpha.
 */
int gala_edge_softmax_bwd_f32(const gala_csr_t *A, const float *alpha, const float *d_alpha,
                              int32_t heads, int32_t mode, float *d_logits, void *stream);

/*
 * Fused GAT aggregation (one pass over the edges):
 *   s = LeakyReLU_slope(aL[row,h] + aR[col,h]);  alpha = edge-softmax(s) (mode);
 *   Y[row, h*D:(h+1)*D] = sum_e alpha[e,h] * X[col, h*D:(h+1)*D],  F = heads*D.
 * alpha_out (nullable) receives alpha for the backward pass.
 * Replaces the forward chain edge_sddvv -> LeakyReLU -> softmax autograd -> weighted
 * aggregate_node_mul_sum_call (common.h:622-894).
 */
int gala_gat_fwd_f32(const gala_csr_t *A, const float *aL, const float *aR, const float *X,
                     int64_t ldx, int32_t F, int32_t heads, float slope, int32_t mode, float *Y,
                     int64_t ldy, float *alpha_out, void *stream);

/*
 * Fused GAT backward over the edges of A (the forward pattern), per head h:
 *   d_alpha[e] = <dY[row, hD:(h+1)D], X[col, hD:(h+1)D]>;  sds = alpha*d_alpha;
 *   acc = S*eps + sum_row sds;  ds = sds - alpha*acc;
 *   dz = ds if aL[row,h]+aR[col,h] > 0 else ds*slope       (LeakyReLU backward);
 *   d_aL[row,h] = S*eps + sum_row dz                         (eps = 1e-12 REF, 0 FIXED).
 * d_logit (nullable in REF mode, required in FIXED mode) receives dz per (edge, head);
 * REF mode computes the row sum of dz as sum(m*sds) - acc*sum(m*alpha), m the LeakyReLU
 * slope factor, in the same single pass.  Replaces the backward chain edge_sddmm ->
 * softmax backward -> LeakyReLU backward -> node_spmv_backward_of_sddmm
 * (cuda.h:505-524,808-845; common.h:622-675,791-799,835-894) in one kernel.  Requires
 * heads | 64 and D/VEC a power of two when heads > 1 (else GALA_ERR_UNSUPPORTED).
 */
int gala_gat_bwd_f32(const gala_csr_t *A, const float *aL, const float *aR, const float *X,
                     int64_t ldx, const float *dY, int64_t lddy, int32_t F, int32_t heads,
                     float slope, int32_t mode, const float *alpha, float *d_logit, float *d_aL,
                     void *stream);

/*
 * The same fused forward / backward with the source logit recomputed from the aggregated
 * rows instead of read from aR: aR[j] = <X[j, 0:F], wR[0:F]> + bR[0] (bR nullable = 0).
 * This is the DSL's GAT layer, where attnR = dsl.nn.ffn(res, out=1) is a Linear of the
 * very `res` that the layer aggregates (tests/GALA-DSL/gat/Products/h100.txt:7-11): the
 * kernels gather X[col] anyway, so the per-edge aR[col] read disappears.  One head.
 * gala_gat_bwd_attn_f32 is REF mode (d_aL = d_aR, no per-edge output).  The gradients
 * of wR / bR / X through aR follow from d_aR on the caller's side (dense, per row).
 */
int gala_gat_fwd_attn_f32(const gala_csr_t *A, const float *aL, const float *wR,
                          const float *bR, const float *X, int64_t ldx, int32_t F, float slope,
                          int32_t mode, float *Y, int64_t ldy, float *alpha_out, void *stream);
int gala_gat_bwd_attn_f32(const gala_csr_t *A, const float *aL, const float *wR,
                          const float *bR, const float *X, int64_t ldx, const float *dY,
                          int64_t lddy, int32_t F, float slope, const float *alpha, float *d_aL,
                          void *stream);

/*
 * The fused GAT forward / backward, general form (q_out may also be given with alpha_out
 * NULL: then only Y and q are written, for gala_gat_bwd_fused_f32):
 *   - the source logit comes from aR [n_cols, heads], or (aR == NULL) is recomputed from
 *     the gathered rows per head: aR[j,h] = <X[j, hD:(h+1)D], wR[hD:(h+1)D]> + bR[h]
 *     (bR nullable = 0; the multi-head GAT layer's attnR = a_r^h . res_j^h);
 *   - the attention output is either alpha (q_out == NULL, as gala_gat_fwd_f32) or, in
 *     REF mode, FACTORED: alpha_out receives p[e,h] = min(exp(s), 1e12) and q_out[r,h] =
 *     1 / (S*1e-12 + sum_row p), so alpha = p * q (rounded) -- bit-identical to the
 *     materialised alpha -- without the normalisation pass over the edges.  The backward
 *     takes the same pair (q != NULL), and the dX SpMM reads it through
 *     gala_csr_t.val = p, val_row_scale = q.
 * Several heads need D = F/heads a multiple of the vector width with D/VEC a power of two
 * for the recompute (else GALA_ERR_UNSUPPORTED).  Replaces the same chains as
 * gala_gat_fwd_f32 / gala_gat_bwd_f32.
 */
/* mode flag of gala_gat_fwd_ex_f32 (REF only, q_out required, alpha_out NULL): a PARTIAL
 * forward over one column range of the graph -- Y[r] = sum_e p_e X[col_e] unnormalised and
 * q_out[r,h] = sum_e p_e (no 1e-12) -- whose partial rows and sums the caller adds over the
 * column ranges (the vertex-cut GAT, gala/vertex_cut.py) before Y = Y_sum / (sum + 1e-12). */
#define GALA_GAT_PARTIAL 0x10
int gala_gat_fwd_ex_f32(const gala_csr_t *A, const float *aL, const float *aR, const float *wR,
                        const float *bR, const float *X, int64_t ldx, int32_t F, int32_t heads,
                        float slope, int32_t mode, float *Y, int64_t ldy, float *alpha_out,
                        float *q_out, void *stream);
int gala_gat_bwd_ex_f32(const gala_csr_t *A, const float *aL, const float *aR, const float *wR,
                        const float *bR, const float *X, int64_t ldx, const float *dY,
                        int64_t lddy, int32_t F, int32_t heads, float slope, int32_t mode,
                        const float *alpha, const float *q, float *d_logit, float *d_aL,
                        void *stream);

/*
 * REF-mode GAT backward with the attention RECOMPUTED and dX fused (square graph whose
 * backward pattern is the forward one -- the undirected graphs the reference runs,
 * cuda.h:1253-1257).  Per row r and head h, over the edges e = (r, c):
 *   alpha = fl(min(exp(LeakyReLU(aL[r,h] + aR[c,h])), 1e12) * q[r,h])   (q: the forward's
 *           q_out; aR or its per-head recompute from X as in gala_gat_fwd_ex_f32)
 *   dX[r, head h] = sum_e alpha * dY[c, head h]       (bit-identical to gala_spmm_f32 over
 *                                                      the materialised alpha)
 *   d_aL[r,h] as gala_gat_bwd_f32 in REF mode (= d_aR), within fp32 rounding.
 * With this the forward need not output alpha at all (gala_gat_fwd_ex_f32 with q_out and
 * alpha_out NULL).  Replaces the backward of the emitted GAT layer: the weighted SpMM
 * <K>_AutoGrad::backward (common.h:835-894) plus the edge chain of gala_gat_bwd_f32.
 * Several heads need D/VEC a power of two (else GALA_ERR_UNSUPPORTED).
 */
int gala_gat_bwd_fused_f32(const gala_csr_t *A, const float *aL, const float *aR,
                           const float *wR, const float *bR, const float *X, int64_t ldx,
                           const float *dY, int64_t lddy, int32_t F, int32_t heads, float slope,
                           const float *q, float *dX, int64_t lddx, float *d_aL, void *stream);

/*
 * REF-mode GAT with ROW STATISTICS (square pattern whose backward pattern is the forward
 * one, as gala_gat_bwd_fused_f32).  The reference's d_aL row sum (common.h:622-675,
 * 791-799, 835-894) is, per row r and head h, with m_e = 1 if aL[r,h] + aR[c_e,h] > 0 else
 * slope (the LeakyReLU factor):
 *   sum_e m_e ds_e = sum_e m_e alpha_e d_alpha_e - acc * sum_e m_e alpha_e,
 *   acc = S*eps + sum_e alpha_e d_alpha_e,       d_alpha_e = <dY[r], X[c_e]>  (per head)
 * and both edge sums regroup into row-local dot products with rows the forward can build
 * from the X rows it gathers anyway:
 *   sum_e alpha_e d_alpha_e     = <dY[r], Y[r]>,   Y[r]  = sum_e alpha_e X[c_e]
 *   sum_e m_e alpha_e d_alpha_e = <dY[r], Ym[r]>,  Ym[r] = sum_e m_e alpha_e X[c_e]
 * So the forward writes Ym (ld ldym) and sma[r,h] = sum_e m_e alpha_e beside Y and q, and
 * the backward gathers dY[col] only (for dX) instead of dY[col] and X[col].  Equal to the
 * reference within fp32 rounding (the sums are regrouped); dX is bit-identical to
 * gala_gat_bwd_fused_f32's.
 *
 * gala_gat_fwd_stats_f32: Y, q_out as gala_gat_fwd_ex_f32 in REF mode with alpha_out NULL,
 * plus Ym, sma.  aR or (aR NULL) its per-head recompute from X (wR, bR); aR_out (nullable)
 * then receives every row's recomputed source logit, bit-identical to the per-edge
 * recompute, for the backward.  p_out (nullable, [nnz, heads]) receives the edges' exp
 * terms p = min(exp(s), 1e12), as gala_gat_fwd_ex_f32's factored output; the backward
 * then reads them in edge order instead of gathering aR[col] (cheaper for narrow rows,
 * where that 4-B random read costs a cache line per edge next to a 1-2 line row gather).
 * Several heads need D/VEC a power of two (else
 * GALA_ERR_UNSUPPORTED; the caller then takes gala_gat_fwd_ex_f32 + gala_gat_bwd_fused_f32).
 * gala_gat_bwd_stats_f32: dX[r] = sum_e alpha_e dY[c_e] (alpha = fl(min(exp(LeakyReLU(
 * aL + aR)), 1e12) * q) from aR, or fl(p * q) when the forward's p is given (aR may then be
 * NULL)) and d_aL[r,h] = (<dY,Ym>_h - (S*eps + <dY,Y>_h) *
 * sma[r,h]) + S*eps (= d_aR in REF mode), eps = 1e-12.
 */
int gala_gat_fwd_stats_f32(const gala_csr_t *A, const float *aL, const float *aR, const float *wR,
                           const float *bR, const float *X, int64_t ldx, int32_t F, int32_t heads,
                           float slope, float *Y, int64_t ldy, float *q_out, float *Ym,
                           int64_t ldym, float *sma, float *aR_out, float *p_out, void *stream);
int gala_gat_bwd_stats_f32(const gala_csr_t *A, const float *aL, const float *aR, const float *p,
                           const float *dY, int64_t lddy, int32_t F, int32_t heads, float slope,
                           const float *q, const float *Y, int64_t ldy, const float *Ym,
                           int64_t ldym, const float *sma, float *dX, int64_t lddx, float *d_aL,
                           void *stream);
/*
 * The same pair over a gathered feature table (a row partition's halo, gala/dist.py
 * HaloGat): the pattern's columns index the table (n_cols >= n_rows), so a row is no longer
 * its own column.  gala_gat_fwd_stats_ex_f32: self_col[r] = the table column of row r's own
 * vertex (NULL: r itself, square pattern), aR_out column-indexed ([n_cols, heads], written at
 * the own columns).  gala_gat_bwd_stats_ex_f32: dY is the gathered table (dY[c] per edge),
 * dY_rows the rows' own dY (row r at dY_rows + r*lddy, e.g. the table's own block; NULL:
 * dY itself, square pattern).  Results equal the one-GPU pair's on the same rows bit for bit.
 */
int gala_gat_fwd_stats_ex_f32(const gala_csr_t *A, const float *aL, const float *aR, const float *wR,
                              const float *bR, const float *X, int64_t ldx, int32_t F, int32_t heads,
                              float slope, float *Y, int64_t ldy, float *q_out, float *Ym, int64_t ldym,
                              float *sma, const int32_t *self_col, float *aR_out, float *p_out, void *stream);
int gala_gat_bwd_stats_ex_f32(const gala_csr_t *A, const float *aL, const float *aR, const float *p,
                              const float *dY, int64_t lddy, const float *dY_rows, int32_t F, int32_t heads,
                              float slope, const float *q, const float *Y, int64_t ldy, const float *Ym,
                              int64_t ldym, const float *sma, float *dX, int64_t lddx, float *d_aL,
                              void *stream);
/*
 * gala_gat_bwd_stats_linear_f32: gala_gat_bwd_stats_ex_f32 (a square pattern with dY_rows
 * NULL, or a gathered dY table with the rows' own dY_rows, as HaloGat.backward runs it)
 * with the source logit's per-head Linear (aR = X wR + bR, the DSL's attnR = ffn(res, out=1),
 * gala_head_attn_f32) folded into the dX store: dX[r, f] += d_aL[r, head(f)] * wR[f], REF's
 * d_aR = d_aL (common.h:835-894 on the undirected pattern), with the product-then-sum
 * roundings of gala_head_attn_bwd_f32 -- bit-identical to that pass after the statistics
 * backward, without re-reading and re-writing dX.
 */
int gala_gat_bwd_stats_linear_f32(const gala_csr_t *A, const float *aL, const float *aR, const float *p,
                                  const float *dY, int64_t lddy, const float *dY_rows, int32_t F, int32_t heads,
                                  float slope, const float *q, const float *Y, int64_t ldy, const float *Ym,
                                  int64_t ldym, const float *sma, const float *wR, float *dX, int64_t lddx,
                                  float *d_aL, void *stream);
/*
 * gala_gat_fwd_partial_stats_f32: gala_gat_fwd_stats_f32 over the columns one rank of a
 * vertex cut holds, every output unnormalised so that the rows' owners add the ranks'
 * partials before they divide (GALA_GAT_PARTIAL of gala_gat_fwd_ex_f32, plus the row
 * statistics):  U[r] = sum_e p_e X[c_e],  sums[r,h] = sum_e p_e,  Um[r] = sum_e m_e p_e X[c_e],
 * msums[r,h] = sum_e m_e p_e  (p_e = min(exp(LeakyReLU(aL[r] + aR[c_e])), 1e12), m_e the
 * LeakyReLU factor).  The owner then forms q = 1 / (sum_p sums + S*1e-12), Y = q*U,
 * Ym = q*Um, sma = q*msums: the inputs gala_gat_bwd_stats_f32 takes.  The REF softmax
 * subtracts no row maximum (common.h:760-773), so partial sums simply add.  Replaces the
 * torch softmax composition of common.h:735-810 for a row whose edges span several GPUs.
 */
int gala_gat_fwd_partial_stats_f32(const gala_csr_t *A, const float *aL, const float *aR, const float *wR,
                                   const float *bR, const float *X, int64_t ldx, int32_t F, int32_t heads,
                                   float slope, float *U, int64_t ldu, float *sums, float *Um, int64_t ldum,
                                   float *msums, void *stream);
/*
 * gala_gat_fwd_partial_stats_ex_f32: the same, and with the source logits recomputed (aR
 * NULL, wR given) also the rank's own vertices' logits: a vertex cut's rows are destination
 * rows and its columns the rank's vertices, so self_col[r] names the column of row r's own
 * vertex (-1 when the rank does not own it).  aR_out[self_col[r]*heads + h] is the logit the
 * kernel forms for that column's edges, taken from the row's self-loop edge (else from the
 * vertex's X row), bit for bit: the backward's alpha uses exactly the forward's logits.
 * aR_out needs self_col (and the recompute).
 */
int gala_gat_fwd_partial_stats_ex_f32(const gala_csr_t *A, const float *aL, const float *aR, const float *wR,
                                      const float *bR, const float *X, int64_t ldx, int32_t F, int32_t heads,
                                      float slope, float *U, int64_t ldu, float *sums, float *Um, int64_t ldum,
                                      float *msums, const int32_t *self_col, float *aR_out, void *stream);

/*
 * gala_gat_fwd_continue_f32: the REF forward (Ym NULL) or row-statistics forward (Ym given)
 * of rows whose edges were split over two column ranges, continued from the unnormalised
 * partials of the first range (gala_gat_fwd_ex_f32 / _partial_stats_ex_f32 with
 * GALA_GAT_PARTIAL): each row's state starts at U0 = sum p X, S0 = sum p (and Um0 = sum m p X,
 * M0 = sum m p) and takes this pattern's edges, then Y = q (U0 + ...), q = 1/(S0 + ... + 1e-12),
 * Ym, sma as gala_gat_fwd_stats_f32.  The inputs may alias the outputs (Y = U0, q_out = S0,
 * Ym = Um0, sma = M0).  flags GALA_GAT_PARTIAL (else 0): the sums are continued but left
 * unnormalised (Y = U0 + sum p X, q_out = the raw sum, ...), for one more range after this
 * one (a halo that lands in row chunks).  Used by a row partition whose own-column edges run while the halo
 * rows are in flight (gala/dist.py HaloGatOverlap); no reference counterpart (the split of
 * the sums is this framework's, common.h:760-773 has the REF sums).  The sums are grouped
 * per range, so the results match the one-pass forward to fp32 rounding.
 */
int gala_gat_fwd_continue_f32(const gala_csr_t *A, const float *aL, const float *aR, const float *wR,
                              const float *bR, const float *X, int64_t ldx, int32_t F, int32_t heads,
                              float slope, int32_t flags, const float *U0, int64_t ldu0, const float *S0, const float *Um0,
                              int64_t ldum0, const float *M0, float *Y, int64_t ldy, float *q_out, float *Ym,
                              int64_t ldym, float *sma, void *stream);

/*
 * Per-head attention logits of the multi-head GAT layer (galac gat_heads: the DSL's
 * attnL / attnR = dsl.nn.ffn(res, out=1) applied per head, a torch::nn::Linear in the
 * reference, common.h:1188-1242):
 *   out[r*heads + h] = <X[r, hD:(h+1)D], w[hD:(h+1)D]> + b[h]     (b nullable; D = F/heads)
 * (an fma chain over each lane's vector, then a fixed butterfly over the head's lanes:
 * deterministic, within fp32 rounding of the sequential sum).  gala_head_attn_bwd_f32 is
 * its input gradient:
 *   dX[r, hD+d] = g[r*heads + h] * w[hD+d]      (accumulate != 0: dX += ..., one rounding
 *                                                each for the product and the sum)
 * The weight / bias gradients are gala_dense_grad_f32 with M = heads (the block diagonal
 * of its [heads, F] result).
 */
int gala_head_attn_f32(int64_t n_rows, int32_t F, int32_t heads, const float *X, int64_t ldx,
                       const float *w, const float *b, float *out, void *stream);
int gala_head_attn_bwd_f32(int64_t n_rows, int32_t F, int32_t heads, const float *g, const float *w,
                           float *dX, int64_t lddx, int32_t accumulate, void *stream);

/*
 * The multi-head GAT layer in INPUT space (ABI 5; config 3's layer 1).  Replaces, for a layer
 * whose aggregated rows are a Linear of a narrower input (the tests/GALA-DSL/gat programs: res =
 * dsl.nn.ffn(G.node.feats, out=hs); attnL / attnR = dsl.nn.ffn(res, out=1); softmax;
 * res = aggregate_fn(G.graphs, res)), the chain FFN_OP (common.h:1188-1242) -> the two
 * attention Linears (common.h:1248-1260) -> the REF edge chain K5-K8 + the weighted
 * aggregation (cuda.h:286-358,505-562,679-698; common.h:735-810) and its REF backward
 * (common.h:835-894: dX = A_alpha dY with the forward alpha, the K9 / softmax / K7 chain):
 * per head h, with W_h the [D, fin] block of the Linear and Xin_ext = [Xin, 1], W_ext = [W, b],
 *     aL = Xin uL^T + cL, aR = Xin uR^T + cR  (uL_h = W_h^T wL_h, cL_h = b_h . wL_h + bL_h)
 *     Y_h[r]  = q_h[r] (sum_e p_e,h Xin_ext[c_e]) W_ext,h^T,   q = 1 / (1e-12 + sum_e p_e)
 *     p = min(exp(LeakyReLU(aL[r] + aR[c])), 1e12)
 * so the edges gather the fin-float input row instead of the H*D-float Linear output.
 *   gala_gat_in_prep_f32: Xext [n][128] (16-B aligned) = the extended rows: Xin's fin <= 100
 *     features, the ones column, aL / aR (u [2H][fin]: uL rows then uR rows; c [2H]).  Every
 *     forward (aL / aR follow the weights).
 *   order (nullable; else A->split->row_order, else row-id order): the order rows (columns) are
 *     taken in, eight per workgroup phase -- a descending-degree order (gala_host_row_order)
 *     gives the eight rows of a phase equal lengths.
 *   gala_gat_in_fwd_f32: Y, Ym [n][ldy] (Ym = the m-weighted aggregate, m = 1 or slope by the
 *     logit's sign), q, sma [n][H] (the row statistics of gala_gat_fwd_stats_f32); writes q
 *     into Xext too (the backward reads it there).  W [H*D][ldw], b [H*D] nullable.
 *   gala_gat_in_bwd_f32: AT = the TRANSPOSED pattern of A (A itself for the symmetric graphs
 *     of undirected programs).  d_aL [n][H] (REF: d aR = d aL) and
 *     M [H][D][fin+1] = sum_r dX[r]^T Xin_ext[r] with dX the REF aggregation backward -- the
 *     FFN's weight gradient through the aggregation (column fin: its bias gradient); the
 *     attention Linears' terms follow from G = d_aL^T Xin_ext (gala_dense_grad_f32):
 *     dW_h += (wL_h + wR_h) G_h, d wL_h = d wR_h = W_ext,h G_h, d bL = d bR = sum d_aL.
 *     ws: gala_gat_in_bwd_workspace(heads) bytes.
 *   flags GALA_GAT_IN_RELU (both calls): the program's NON_LNR_OP_RELU after the layer fused --
 *     the forward stores relu(Y) (NaN kept, as torch::relu) and the backward takes the
 *     gradient of relu(Y), masked by relu(Y) > 0 (torch's threshold_backward); the d_aL dots
 *     <dY, Y> are then the same sums over relu(Y).
 * Limits (else GALA_ERR_UNSUPPORTED, callers keep the statistics pair): fin <= 100, heads
 * <= 8, D in {4, 8, 16, 32}, one segment, a square pattern, no hub rows in A->split (a hub
 * row would be one wave's serial walk).  Sums are regrouped (the matrix cores sum four edges
 * per step; the input-space association): fp32 rounding of the reference, checked at 1e-4.
 */
int gala_gat_in_prep_f32(int64_t n, int32_t fin, const float *Xin, int64_t ldxin, int32_t heads,
                         const float *u, const float *c, float *Xext, void *stream);
#define GALA_GAT_IN_RELU 1   /* the layer's ReLU fused: Y = relu(.) forward, dY masked by Y > 0 backward */
int gala_gat_in_fwd_f32(const gala_csr_t *A, const int32_t *order, int32_t fin, int32_t heads, int32_t D, float slope,
                        float *Xext, const float *W, int64_t ldw, const float *b, float *Y, float *Ym,
                        int64_t ldy, float *q, float *sma, int32_t flags, void *stream);
int64_t gala_gat_in_bwd_workspace(int32_t heads);
int gala_gat_in_bwd_f32(const gala_csr_t *AT, const int32_t *order, int32_t fin, int32_t heads, int32_t D, float slope,
                        const float *Xext, const float *dY, const float *Y, const float *Ym,
                        int64_t ldy, const float *sma, float *daL, float *M, void *ws,
                        int64_t ws_bytes, int32_t flags, void *stream);
/* T mode (round 6; symmetric A only -- A equal to its transpose, which the caller checks):
 *   gala_gat_in_fwd_t_f32: gala_gat_in_fwd_f32 that first sums q for every row (a pass over the
 *     aR of each row's columns, in CSR order) and then, in the same walk as Y, forms the
 *     backward's per-column aggregates T [n][896] (16-B aligned; 3.5 KB per row) -- so
 *     gala_gat_in_bwd_t_f32 reads T and dY instead of gathering the extended rows again.
 *   gala_gat_in_bwd_t_f32: gala_gat_in_bwd_f32's outputs (d_aL, M) from T; no graph. */
int gala_gat_in_fwd_t_f32(const gala_csr_t *A, const int32_t *order, int32_t fin, int32_t heads, int32_t D,
                          float slope, float *Xext, const float *W, int64_t ldw, const float *b, float *Y,
                          float *Ym, int64_t ldy, float *q, float *sma, int32_t flags, float *T, void *stream);
int gala_gat_in_bwd_t_f32(int64_t n_rows, const int32_t *order, int32_t fin, int32_t heads, int32_t D,
                          const float *T, const float *dY, const float *Y, const float *Ym, int64_t ldy,
                          const float *sma, float *daL, float *M, void *ws, int64_t ws_bytes, int32_t flags,
                          void *stream);

/* dst[i*heads + h] = src[perm[i]*heads + h]  (edge-value permutation for transposed graphs) */
int gala_edge_permute_f32(const int32_t *perm, const float *src, int64_t n, int32_t heads,
                          float *dst, void *stream);

/* ---- host-side graph layout (HOST pointers, OpenMP) --------------------------------- */

/*
 * COO -> CSR: counting sort by src, then cols ascending inside each row, duplicates
 * kept (CSRCMatrix::build, csrc_matrix.h:148-376; count_atomic / count_sort_place_*,
 * sort_range*arr, src/utils/mtx_sort.h:52-174,683-761).  perm_out (nullable) receives the
 * input index of every CSR edge (stable: ties keep input order).
 */
int gala_host_csr_build(int64_t n_rows, int64_t n_cols, int64_t nnz, const int32_t *src,
                        const int32_t *dst, int32_t *rowptr_out, int32_t *col_out,
                        int32_t *perm_out);

/*
 * Column breakpoints {0, c, 2c, ..., n_cols} (static_ord_col_breakpoints,
 * tiling.h:1594-1608).  Writes at most max_out entries; returns the count (>=2) or <0.
 */
int64_t gala_host_col_breakpoints(int64_t n_cols, int64_t cols_per_partition,
                                  int32_t *out, int64_t max_out);

/*
 * Column tiling into the relative-offset segment layout (ord_col_tiling_torch,
 * tiling.h:222-283).  breakpoints has n_seg+1 entries; out_rowptr [(n_rows+1)*n_seg],
 * out_col/out_val [nnz], out_bounds [2*n_seg].  val / out_val may be NULL.
 */
int gala_host_col_tile(int64_t n_rows, const int32_t *rowptr, const int32_t *col,
                       const float *val, int32_t n_seg, const int32_t *breakpoints,
                       int32_t *out_rowptr, int32_t *out_col, float *out_val,
                       int32_t *out_bounds);

/*
 * Deterministic data sampling: every row keeps nsamp edges j = (ra*ji+rb) mod deg,
 * sorted (inplace_sample_graph_ab, tiling.h:454-508).  out_rowptr [n_rows+1],
 * out_col/out_val [n_rows*nsamp].  A row with deg 0 is GALA_ERR_GRAPH (the reference
 * divides by zero there).
 */
int gala_host_sample_ab(int64_t n_rows, const int32_t *rowptr, const int32_t *col,
                        const float *val, int32_t nsamp, int32_t ra, int32_t rb,
                        int32_t *out_rowptr, int32_t *out_col, float *out_val);

/*
 * Split plan of a CSR (gala_split_plan_t): rows with deg > threshold, chunks of `chunk`
 * edges.  Two-call pattern: with rows/row_chunk0/chunk_row NULL it only writes the counts
 * (*n_rows_split, *n_chunks); then call again with arrays of those sizes (+1 for
 * row_chunk0).
 */
int gala_host_split_plan(int64_t n_rows, const int32_t *rowptr, int32_t threshold, int32_t chunk,
                         int32_t *rows, int32_t *row_chunk0, int32_t *chunk_row,
                         int64_t *n_rows_split, int64_t *n_chunks);

/*
 * The hub-row threshold every caller uses for a graph of n_rows rows and nnz edges:
 * max(1024, 8 * ceil(nnz / n_rows)).  One definition for the Python layer, the C++ operator
 * mirror and the partitioners, so a partition of a graph splits exactly the rows the whole
 * graph splits (bit-identical multi-GPU results).  Returns < 0 on negative sizes.
 */
int32_t gala_host_split_threshold(int64_t n_rows, int64_t nnz);

/*
 * Row schedule for skewed graphs: order[] = the rows sorted by descending degree, ties by
 * row id (a counting sort up to degree 4096, the rows above it sorted exactly).  Degree-aware
 * row binning: rows that share a wavefront then have similar lengths; and for
 * any threshold the rows longer than it are exactly the order's first entries (the REF-order
 * hub kernel's contract, gala_split_plan_t.row_order).
 */
int gala_host_row_order(int64_t n_rows, const int32_t *rowptr, int32_t *order);

/*
 * Transpose a CSR (n_seg == 1): out_rowptr [n_cols+1], out_col [nnz], perm [nnz] with
 * out edge k == in edge perm[k] (used by the FIXED-mode backward; the reference reuses
 * the forward graph, cuda.h:1253-1257).
 */
int gala_host_csr_transpose(int64_t n_rows, int64_t n_cols, const int32_t *rowptr,
                            const int32_t *col, int32_t *out_rowptr, int32_t *out_col,
                            int32_t *perm);

/*
 * Deterministic synthetic graphs (counter-based hash RNG, thread-count independent):
 *   kind 0: uniform random symmetric edges + one self loop per vertex;
 *   kind 1: R-MAT (a=0.57,b=0.19,c=0.19; src/utils/generator.h:37-118) symmetrised
 *           + self loops;
 *   kind 2: banded: the two ends of an edge at most min(8192, max(16, n/256)) ids apart (locality,
 *           the shape a locality-preserving vertex order gives), symmetrised + self loops.
 * n_undirected undirected edges -> 2*n_undirected + n vertices directed COO entries
 * written to src/dst (capacity 2*n_undirected + n).
 */
int gala_host_gen_graph(int32_t kind, int64_t n, int64_t n_undirected, uint64_t seed,
                        int32_t *src, int32_t *dst);

/*
 * Matrix Market graphs: the reference's readSM -> MtxIO::readMtx / readMM
 * (src/utils/common.h:397-416, src/utils/mtx_io.h:199-499), coordinate format.
 * gala_host_mtx_info reads the header and the size line:
 *   field     0 pattern, 1 integer, 2 real, 3 double (complex: GALA_ERR_UNSUPPORTED)
 *   symmetry  0 general, 1 symmetric, 2 skew-symmetric (hermitian: GALA_ERR_UNSUPPORTED)
 *   capacity  COO entries gala_host_mtx_read may write: nnz, twice that when symmetric.
 * "array" (dense) files are GALA_ERR_UNSUPPORTED; a missing or malformed file is
 * GALA_ERR_INVALID_ARG.
 * gala_host_mtx_read writes the entries 0-based in file order; an off-diagonal entry of a
 * (skew-)symmetric file is followed by its mirror with the SAME value (the reference does
 * not negate skew-symmetric mirrors).  As in the reference, the entry lines are read while
 * each ends in a newline: a last line without one is not read.  vals may be NULL; for a
 * pattern file it receives 1.0f (the reference leaves pattern values unallocated).
 * Indices outside [1, n] are GALA_ERR_GRAPH (the reference does not check them).
 * *count_out = entries written.
 */
int gala_host_mtx_info(const char *path, int64_t *n_rows, int64_t *n_cols, int64_t *nnz, int32_t *field,
                       int32_t *symmetry, int64_t *capacity);
int gala_host_mtx_read(const char *path, int32_t *rows, int32_t *cols, float *vals, int64_t capacity,
                       int64_t *count_out);

/*
 * A dense Matrix Market "array" file (features; the reference's readDM without RNPY,
 * src/utils/common.h:146-183 -> MtxIO::readMM's array branch, mtx_io.h:316-363):
 * gala_host_mtx_dense_info gives its shape, gala_host_mtx_read_dense writes it row-major into
 * out[n_rows * n_cols] (the file lists it column by column).  Integer, real and double
 * fields, general symmetry only (else GALA_ERR_UNSUPPORTED, as the reference refuses them);
 * entries the file does not hold (it ends early, or its last line lacks a newline, which
 * the reference then does not read) are set to 0.  *count_out = entries read.
 */
int gala_host_mtx_dense_info(const char *path, int64_t *n_rows, int64_t *n_cols);
int gala_host_mtx_read_dense(const char *path, float *out, int64_t n_rows, int64_t n_cols, int64_t *count_out);

/*
 * FFN (torch Linear) gradients of a tall-skinny node matrix: dW[m,k] = sum_n dY[n,m]
 * X[n,k] ([M,K] row-major, the Linear weight layout) and, if db != NULL, db[m] =
 * sum_n dY[n,m].  accumulate != 0 adds into dW / db.  The rows are split into chunks
 * whose partial tiles go to `workspace` (gala_dense_grad_workspace bytes), then summed
 * in chunk order: deterministic for given shapes.  Replaces the weight / bias part of
 * the backward of the generated programs' FFN_OP (common.h:1188-1242; torch's generic
 * kernels serve that backward in the reference).
 */
int64_t gala_dense_grad_workspace(int64_t n_rows, int32_t K, int32_t M);
int gala_dense_grad_f32(int64_t n_rows, int32_t K, int32_t M, const float *X, int64_t ldx,
                        const float *dY, int64_t ldy, float *dW, float *db, int32_t accumulate,
                        void *workspace, int64_t workspace_bytes, void *stream);

/*
 * FFN forward on tall-skinny node matrices: Y[n, :] = X[n, 0:K] W^T + b, W [M, K] row-major
 * (a torch Linear weight), b [M] or NULL.  Exact-f32 matrix cores, W^T held in LDS: K * M up
 * to 16384 floats (rounded up to 32-column tiles), else GALA_ERR_UNSUPPORTED (callers use
 * the library GEMM).  Replaces the forward of the generated programs' FFN_OP
 * (common.h:1188-1242, torch::nn::Linear in the reference) and, with W^T, its dX.
 */
int gala_ffn_fwd_f32(int64_t n_rows, int32_t K, int32_t M, const float *X, int64_t ldx,
                     const float *W, const float *b, float *Y, int64_t ldy, void *stream);

/*
 * One level of the training-subgraph transformation (getMaskSubgraphs,
 * tests/common.h:21-110; requested by middle-end.h:39-211 and emitted by
 * codegen/common.h:480-492): out = the rows i with mask[i] > 0 (all their edges, in
 * order), every other row empty; next_mask[i] = max over row i's edges of mask[col]
 * (gSpMM with maxAgg) for the level below.  Two-call pattern: with out_col == NULL only
 * out_rowptr [n_rows+1] is written (its last entry is the nnz to allocate).
 * next_mask may be NULL.
 */
int gala_host_mask_subgraph(int64_t n_rows, const int32_t *rowptr, const int32_t *col,
                            const int32_t *mask, int32_t *out_rowptr, int32_t *out_col,
                            int32_t *next_mask);

#ifdef __cplusplus
}
#endif
#endif /* GALA_HIP_H */
