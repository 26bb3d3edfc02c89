/*
 * gala_cpu.h — C ABI of libgala_cpu.so, the host-CPU backend of GALA's generated
 * programs (the reference's CPU code generator is an empty stub,
 * src/codegen/cpu.h:1-7, and its drivers hard-code the GPU device,
 * tests/gala_inference.cpp:174-175).
 *
 * Every gala_cpu_X has the signature and semantics of gala_X in gala_hip.h, with HOST
 * pointers instead of device pointers; `stream` is accepted and ignored.  The operator
 * mirror (host/gala_torch.cpp) calls these for tensors a program placed on the CPU
 * (`--device cpu`) and the gala_hip.h entry points for tensors on the GPU: the device is
 * the program's explicit choice, never a fallback, and a GPU tensor never reaches this
 * library.
 *
 * Numerics follow gala_hip.h's contract: edges are accumulated sequentially in CSR order
 * per row with the reference's rounding steps, so SpMM / degree / SDDVV / row-scale /
 * row-broadcast are bit-identical to the GPU kernels (and to the reference kernels); the
 * reductions (row-sum, SDDMM, softmax, GAT) keep the reference's sequential order.
 * Parallel over rows with OpenMP.
 */
#ifndef GALA_CPU_H
#define GALA_CPU_H

#include "gala_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

int gala_cpu_spmm_f32(const gala_csr_t *A, const float *X, int64_t ldx, float *Y, int64_t ldy,
                      int32_t F, const float *src_scale, const float *dst_scale, int32_t flags,
                      int32_t nsamp, int32_t ra, int32_t rb, void *stream);
int gala_cpu_spmm_ex_f32(const gala_csr_t *A, const float *X, int64_t ldx, float *Y, int64_t ldy,
                         int32_t F, const float *src_scale, const float *dst_scale, int32_t flags,
                         int32_t nsamp, int32_t ra, int32_t rb, const gala_spmm_epilogue_t *epi,
                         void *stream);
int gala_cpu_row_broadcast_deg_f32(const gala_csr_t *A, int32_t F, const float *X, int64_t ldx, float *Y,
                                   int64_t ldy, void *stream);
int gala_cpu_degree_f32(const gala_csr_t *A, float *deg, float power, int32_t flags,
                        int32_t nsamp, void *stream);
int gala_cpu_row_broadcast_f32(int64_t n_rows, int32_t F, const float *scale, const float *X,
                               int64_t ldx, float *Y, int64_t ldy, void *stream);
int gala_cpu_row_scale_relu_f32(int64_t n_rows, int32_t F, const float *act, const float *pre,
                                const float *X, int64_t ldx, float *Y, int64_t ldy, void *stream);
int gala_cpu_relu_scale_backward_f32(int64_t n_rows, int32_t F, const float *act, const float *X,
                                     int64_t ldx, const float *G, int64_t ldg, float *dX,
                                     int64_t lddx, void *stream);
int gala_cpu_sddvv_f32(const gala_csr_t *A, const float *a_row, const float *b_col,
                       int32_t heads, int32_t op, float slope, float *out_e, void *stream);
int gala_cpu_row_sum_f32(const gala_csr_t *A, const float *v_e, int32_t heads, float eps,
                         float *out_row, int32_t flags, void *stream);
int gala_cpu_row_scale_f32(const gala_csr_t *A, const float *q_row, int32_t heads,
                           float *v_inout, void *stream);
int gala_cpu_sddmm_dot_f32(const gala_csr_t *A, const float *Ad, int64_t lda, const float *Bd,
                           int64_t ldb, int32_t F, int32_t heads, float *out_e, void *stream);
int gala_cpu_edge_softmax_fwd_f32(const gala_csr_t *A, const float *logits, int32_t heads,
                                  int32_t mode, float *alpha, void *stream);
int gala_cpu_edge_softmax_bwd_f32(const gala_csr_t *A, const float *alpha,
                                  const float *d_alpha, int32_t heads, int32_t mode,
                                  float *d_logits, void *stream);
int gala_cpu_gat_fwd_f32(const gala_csr_t *A, const float *aL, const float *aR, const float *X,
                         int64_t ldx, int32_t F, int32_t heads, float slope, int32_t mode,
                         float *Y, int64_t ldy, float *alpha_out, void *stream);
int gala_cpu_gat_bwd_f32(const gala_csr_t *A, const float *aL, const float *aR, const float *X,
                         int64_t ldx, const float *dY, int64_t lddy, int32_t F, int32_t heads,
                         float slope, int32_t mode, const float *alpha, float *d_logit,
                         float *d_aL, void *stream);
int gala_cpu_gat_fwd_attn_f32(const gala_csr_t *A, const float *aL, const float *wR,
                              const float *bR, const float *X, int64_t ldx, int32_t F,
                              float slope, int32_t mode, float *Y, int64_t ldy, float *alpha_out,
                              void *stream);
int gala_cpu_gat_bwd_attn_f32(const gala_csr_t *A, const float *aL, const float *wR,
                              const float *bR, const float *X, int64_t ldx, const float *dY,
                              int64_t lddy, int32_t F, float slope, const float *alpha,
                              float *d_aL, void *stream);
int gala_cpu_gat_fwd_ex_f32(const gala_csr_t *A, const float *aL, const float *aR,
                            const float *wR, const float *bR, const float *X, int64_t ldx,
                            int32_t F, int32_t heads, float slope, int32_t mode, float *Y,
                            int64_t ldy, float *alpha_out, float *q_out, void *stream);
int gala_cpu_gat_bwd_ex_f32(const gala_csr_t *A, const float *aL, const float *aR,
                            const float *wR, const float *bR, const float *X, int64_t ldx,
                            const float *dY, int64_t lddy, int32_t F, int32_t heads, float slope,
                            int32_t mode, const float *alpha, const float *q, float *d_logit,
                            float *d_aL, void *stream);
int gala_cpu_gat_bwd_fused_f32(const gala_csr_t *A, const float *aL, const float *aR,
                               const float *wR, const float *bR, const float *X, int64_t ldx,
                               const float *dY, int64_t lddy, int32_t F, int32_t heads,
                               float slope, const float *q, float *dX, int64_t lddx,
                               float *d_aL, void *stream);
int gala_cpu_gat_fwd_stats_f32(const gala_csr_t *A, const float *aL, const float *aR,
                               const float *wR, const float *bR, const float *X, int64_t ldx,
                               int32_t F, int32_t heads, float slope, float *Y, int64_t ldy,
                               float *q_out, float *Ym, int64_t ldym, float *sma, float *aR_out,
                               float *p_out, void *stream);
int gala_cpu_gat_bwd_stats_f32(const gala_csr_t *A, const float *aL, const float *aR,
                               const float *p, const float *dY, int64_t lddy, int32_t F, int32_t heads,
                               float slope, const float *q, const float *Y, int64_t ldy,
                               const float *Ym, int64_t ldym, const float *sma, float *dX,
                               int64_t lddx, float *d_aL, void *stream);
int gala_cpu_gat_fwd_stats_ex_f32(const gala_csr_t *A, const float *aL, const float *aR, const float *wR,
                                  const float *bR, const float *X, int64_t ldx, int32_t F, int32_t heads,
                                  float slope, float *Y, int64_t ldy, float *q_out, float *Ym, int64_t ldym,
                                  float *sma, const int32_t *self_col, float *aR_out, float *p_out,
                                  void *stream);
int gala_cpu_gat_fwd_continue_f32(const gala_csr_t *A, const float *aL, const float *aR, const float *wR,
                                  const float *bR, const float *X, int64_t ldx, int32_t F, int32_t heads,
                                  float slope, int32_t flags, const float *U0, int64_t ldu0, const float *S0, const float *Um0,
                                  int64_t ldum0, const float *M0, float *Y, int64_t ldy, float *q_out, float *Ym,
                                  int64_t ldym, float *sma, void *stream);
int gala_cpu_gat_bwd_stats_linear_f32(const gala_csr_t *A, const float *aL, const float *aR, const float *pe,
                                      const float *dY, int64_t lddy, const float *dY_rows, int32_t F, int32_t heads,
                                      float slope, const float *q, const float *Y, int64_t ldy, const float *Ym,
                                      int64_t ldym, const float *sma, const float *wR, float *dX, int64_t lddx,
                                      float *d_aL, void *stream);
int gala_cpu_gat_bwd_stats_ex_f32(const gala_csr_t *A, const float *aL, const float *aR, const float *p,
                                  const float *dY, int64_t lddy, const float *dY_rows, int32_t F,
                                  int32_t heads, float slope, const float *q, const float *Y, int64_t ldy,
                                  const float *Ym, int64_t ldym, const float *sma, float *dX, int64_t lddx,
                                  float *d_aL, void *stream);
int gala_cpu_gat_fwd_partial_stats_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                       const float *wR, const float *bR, const float *X, int64_t ldx,
                                       int32_t F, int32_t heads, float slope, float *U, int64_t ldu,
                                       float *sums, float *Um, int64_t ldum, float *msums, void *stream);
int gala_cpu_gat_fwd_partial_stats_ex_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                          const float *wR, const float *bR, const float *X, int64_t ldx,
                                          int32_t F, int32_t heads, float slope, float *U, int64_t ldu,
                                          float *sums, float *Um, int64_t ldum, float *msums,
                                          const int32_t *self_col, float *aR_out, void *stream);
int gala_cpu_head_attn_f32(int64_t n_rows, int32_t F, int32_t heads, const float *X, int64_t ldx,
                           const float *w, const float *b, float *out, void *stream);
int gala_cpu_head_attn_bwd_f32(int64_t n_rows, int32_t F, int32_t heads, const float *g,
                               const float *w, float *dX, int64_t lddx, int32_t accumulate,
                               void *stream);
int gala_cpu_edge_permute_f32(const int32_t *perm, const float *src, int64_t n, int32_t heads,
                              float *dst, void *stream);
int gala_cpu_ffn_fwd_f32(int64_t n_rows, int32_t K, int32_t M, const float *X, int64_t ldx,
                         const float *W, const float *b, float *Y, int64_t ldy, void *stream);
int64_t gala_cpu_dense_grad_workspace(int64_t n_rows, int32_t K, int32_t M);
int gala_cpu_dense_grad_f32(int64_t n_rows, int32_t K, int32_t M, const float *X, int64_t ldx,
                            const float *dY, int64_t ldy, float *dW, float *db,
                            int32_t accumulate, void *workspace, int64_t workspace_bytes,
                            void *stream);
int gala_cpu_gat_in_prep_f32(int64_t n, int32_t fin, const float *Xin, int64_t ldxin, int32_t heads,
                             const float *u, const float *c, float *Xext, void *stream);
int gala_cpu_gat_in_fwd_f32(const gala_csr_t *A, const int32_t *order, int32_t fin, int32_t heads, int32_t D, float slope,
                            float *Xext, const float *W, int64_t ldw, const float *b, float *Y, float *Ym,
                            int64_t ldy, float *q, float *sma, int32_t flags, void *stream);
int64_t gala_cpu_gat_in_bwd_workspace(int32_t heads);
int gala_cpu_gat_in_bwd_f32(const gala_csr_t *AT, const int32_t *order, int32_t fin, int32_t heads, int32_t D, float slope,
                            const float *Xext, const float *dY, const float *Y, const float *Ym,
                            int64_t ldy, const float *sma, float *daL, float *M, void *ws,
                            int64_t ws_bytes, int32_t flags, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* GALA_CPU_H */
