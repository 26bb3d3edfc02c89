// gala_torch.h — C++/libtorch mirror of the operator API GALA's code generator emits
// into gala.cu, implemented over the C ABI of libgala_hip.so (include/gala_hip.h).
//
// A generated program (or the HIP emitter that replaces src/codegen/cuda.h) calls these
// with exactly the names, argument order and argument meaning of the emitted functions:
//   <aggregate_node_mul_sum[_direct]>_call     src/codegen/cuda.h:441-502 (gala.cu:227-390)
//   gather_forward (cuSPARSE weighted path)      src/codegen/cuda.h:211-279
//   node_spmv_backward_of_sddmm_{nln,eaggr}      src/codegen/cuda.h:565-600, 737-772
//   inplace_softmax_sddvv[_mult]                 src/codegen/cuda.h:601-656
//   edge_sddvv / edge_sddmm                      src/codegen/cuda.h:773-845
//   aggregate_edge_mul / aggregate_edge_mul_dir  src/codegen/cuda.h:870-952
// and the emitted autograd Functions (src/codegen/common.h:622-1084, gala.cu:391-414).
// The `_coarse{C}` suffixes of the emitted names select CUDA launch geometry only; the
// gfx950 kernels pick their own geometry, so every suffix maps to the same function.
//
// Differences from the reference, all deliberate:
//   - errors throw c10::Error (TORCH_CHECK) instead of exit(EXIT_FAILURE);
//   - every kernel runs on the caller's current HIP stream (no leaked per-launch streams);
//   - column-tiled segments are summed in order (no inter-stream race on the output);
//   - the softmax backward does not overwrite the saved forward alpha in place.
#pragma once

#include <torch/torch.h>

#include <memory>
#include <string>
#include <vector>

#include "gala_hip.h"

namespace gala {

// Hub-row split plan of one graph (gala_split_plan_t + the device arrays it points to).
struct SplitState {
    gala_split_plan_t plan{};
    torch::Tensor rows, row_chunk0, chunk_row, row_order, ws;
    // the side stream (torch's pool) and fork / join events of the REF-order hub rows; the
    // events are never destroyed (a plan may outlive the HIP runtime at process exit)
    void *aux_events[2] = {nullptr, nullptr};
    void ensure_workspace(int64_t F);
};
// GALA_SPMM_HUB=chunked selects the fast, reordered hub-row mode (GALA_SPMM_HUB_CHUNKED)
// for every SpMM of the mirror; unset or "exact": the reference's order (the default).
int32_t spmm_hub_flag();
// Builds the plan from the device rowptr (one D2H copy) when some row is longer than
// max(1024, 8 * mean degree) (hub-row split) or the graph is skewed (max degree > 4 x
// mean: descending-degree row order); returns nullptr otherwise or for tiled graphs.
std::shared_ptr<SplitState> make_split_plan(const torch::Tensor &offsets, int segments);

// A column-tiled graph's rows with their segments concatenated (segment 0's edges first,
// each segment's in CSR order: the order every tiled kernel sums in), built once per
// unweighted tiled GPU graph.  The unweighted, unsampled SpMMs of the graph run on it as one
// segment -- bit-identical sums, one rowptr pair per row instead of one per segment, and the
// hub-row / degree-order plan of `split`.  nullptr for untiled, host or malformed graphs.
struct MergedCsr {
    torch::Tensor rowptr, col;
    std::shared_ptr<SplitState> split;
};
std::shared_ptr<MergedCsr> make_merged_csr(const torch::Tensor &offsets, const torch::Tensor &cols,
                                           const torch::Tensor &bounds_host, int segments);

// The transposed pattern of a one-segment slot graph, built on first use (the input-space
// GAT backward walks it): the slot's own tensors when the pattern is symmetric; with the
// descending-degree row orders of both (gala_host_row_order: equal-length rows per phase).
struct PatternT {
    torch::Tensor rowptr, col;
    bool symmetric = false;
    torch::Tensor order, order_t;   // rows of the pattern / of its transpose by descending degree
};

// The generated program's graph slots (codegen/gala.cu:32-43): slot 2*li is layer li's
// forward graph, slot 2*li+1 its backward graph (the same tensors for undirected graphs,
// cuda.h:1253-1257).  `bounds` stay on the host like the reference's total_bounds.
struct GraphSlots {
    std::vector<torch::Tensor> offset_graph, columns_graph, value_graph, bounds;
    std::vector<int> segments;
    std::vector<bool> weighted;
    std::vector<torch::Tensor> transpose_perm;  // optional: edge k of slot == edge perm[k] of forward
    std::vector<std::shared_ptr<SplitState>> split;  // hub-row plans (nullptr: none)
    std::vector<std::shared_ptr<MergedCsr>> merged;  // tiled graphs' merged rows (nullptr: none)
    std::vector<std::shared_ptr<PatternT>> pattern_t;  // transposed patterns (built on first use)
    int64_t nrows = 0;
    int ra = 5, rb = 7;    // kernel-sampling coefficients (common.h:813-833)
    int nsamples = 0;      // 0 = no kernel sampling

    int push(torch::Tensor offsets, torch::Tensor cols, torch::Tensor vals, torch::Tensor bounds,
             int segments, bool weighted);
    void clear();
};
GraphSlots &global_slots();

// ---- emitted free functions ------------------------------------------------------------
torch::Tensor aggregate_node_mul_sum_call(torch::Tensor input_dense, torch::Tensor offset_graph,
                                          torch::Tensor columns_graph, torch::Tensor value_graph,
                                          torch::Tensor bounds = {}, int64_t segments = 1,
                                          bool weighted = false, int64_t nsamples = 0,
                                          int64_t ra = 5, int64_t rb = 7);
torch::Tensor aggregate_node_mul_sum_direct_call(torch::Tensor input_dense,
                                                 torch::Tensor offset_graph,
                                                 torch::Tensor columns_graph,
                                                 torch::Tensor value_graph,
                                                 torch::Tensor bounds = {}, int64_t segments = 1,
                                                 bool weighted = false);
torch::Tensor gather_forward(torch::Tensor input_dense, torch::Tensor offset_graph,
                             torch::Tensor columns_graph, torch::Tensor value_graph);
torch::Tensor node_spmv_backward_of_sddmm_nln(torch::Tensor offset_graph,
                                              torch::Tensor columns_graph,
                                              torch::Tensor value_graph, torch::Tensor bounds,
                                              int64_t nrows, int64_t segments);
torch::Tensor node_spmv_backward_of_sddmm_eaggr(torch::Tensor offset_graph,
                                                torch::Tensor columns_graph,
                                                torch::Tensor value_graph, torch::Tensor bounds,
                                                int64_t nrows, int64_t segments);
torch::Tensor inplace_softmax_sddvv(torch::Tensor row_val, torch::Tensor offset_graph,
                                    torch::Tensor columns_graph, torch::Tensor value_graph,
                                    torch::Tensor bounds, int64_t nrows, int64_t segments);
torch::Tensor inplace_softmax_sddvv_mult(torch::Tensor row_val, torch::Tensor offset_graph,
                                         torch::Tensor columns_graph, torch::Tensor value_graph,
                                         torch::Tensor bounds, int64_t nrows, int64_t segments);
torch::Tensor edge_sddvv(torch::Tensor input_dense1, torch::Tensor input_dense2,
                         torch::Tensor offset_graph, torch::Tensor columns_graph,
                         torch::Tensor value_graph, torch::Tensor bounds, int64_t nrows,
                         int64_t segments);
torch::Tensor edge_sddmm(torch::Tensor input_dense1, torch::Tensor input_dense2,
                         torch::Tensor offset_graph, torch::Tensor columns_graph,
                         torch::Tensor value_graph, torch::Tensor bounds, int64_t nrows,
                         int64_t segments);
torch::Tensor aggregate_edge_mul(torch::Tensor input_dense1, torch::Tensor input_dense2,
                                 torch::Tensor offset_graph, torch::Tensor columns_graph,
                                 torch::Tensor value_graph, torch::Tensor bounds,
                                 int64_t segments);
torch::Tensor aggregate_edge_mul_dir(torch::Tensor input_dense1, torch::Tensor input_dense2,
                                     torch::Tensor offset_graph, torch::Tensor columns_graph,
                                     torch::Tensor value_graph);

// ---- fused ops (no reference counterpart: one kernel for a reference op chain) ---------
// norm * A (norm * X): the GCN aggregation with both ROW_BROADCASTs (gala.cu:442-456)
torch::Tensor gcn_aggregate(torch::Tensor X, torch::Tensor norm, torch::Tensor offset_graph,
                            torch::Tensor columns_graph, torch::Tensor bounds = {},
                            int64_t segments = 1);
torch::Tensor row_broadcast(torch::Tensor scale, torch::Tensor X);
torch::Tensor degree_norm(torch::Tensor offset_graph, torch::Tensor bounds, int64_t segments,
                          double power, torch::Tensor columns_graph = {});

// ---- emitted autograd Functions (apply() wrappers; li = layer index into the slots) ---
torch::Tensor aggregate_node_mul_sum_apply(torch::Tensor input_dense, int64_t li);
torch::Tensor aggregate_node_mul_sum_attn_apply(torch::Tensor input_dense,
                                                torch::Tensor value_graph, int64_t li);
torch::Tensor aggregate_edge_sum_apply(torch::Tensor input_dense1, torch::Tensor input_dense2,
                                       int64_t li);
torch::Tensor non_lnr_op_softmax_apply(torch::Tensor value_graph, int64_t li);
// post * A (pre * X) with autograd on slot 2li (backward: pre * A_b (post * dY) on slot
// 2li+1); pre / post may be undefined.  Honours the slot's weights and kernel sampling.
torch::Tensor gcn_aggregate_apply(torch::Tensor X, torch::Tensor pre, torch::Tensor post,
                                  int64_t li);
// The same with the ReLU prologue of the next layer fused in front: post * A (pre *
// relu(act * X)); act / pre / post may be undefined.  Forward and backward are
// bit-identical to torch::relu(act * X) followed by gcn_aggregate_apply.
torch::Tensor gcn_aggregate_relu_apply(torch::Tensor X, torch::Tensor act, torch::Tensor pre,
                                       torch::Tensor post, int64_t li);
// FFN_OP: X W^T + b (at::linear's forward) whose weight / bias gradients run on
// gala_dense_grad_f32; bias may be undefined.
torch::Tensor ffn_apply(torch::Tensor X, torch::Tensor weight, torch::Tensor bias);
// Fused GAT aggregation with autograd (mode GALA_SOFTMAX_REF reproduces the reference's
// forward and backward chain, GALA_SOFTMAX_FIXED the mathematically correct gradients,
// using the slot's transposed graph).
torch::Tensor gat_aggregate_apply(torch::Tensor attn_l, torch::Tensor attn_r, torch::Tensor X,
                                  int64_t li, double slope, int64_t mode);
// the same layer with attn_r recomputed inside the kernels from the rows they gather (the
// DSL's attnR = dsl.nn.ffn(res, out=1) of the aggregated res).  One head: attn_r = X
// attn_r_weight^T + attn_r_bias; H heads (attn_l [N, H], galac gat_heads(H)): per head h,
// attn_r[:, h] = X[:, head h] . attn_r_weight[head h] + attn_r_bias[h].
torch::Tensor gat_aggregate_ffn_apply(torch::Tensor attn_l, torch::Tensor X, torch::Tensor attn_r_weight,
                                      torch::Tensor attn_r_bias, int64_t li, double slope,
                                      int64_t mode);

// Multi-head attention vectors (galac gat_heads(H)): weight [1, F] holds one vector of D =
// F/H entries per head, bias [H].  Initialised like H Linear(D, 1) layers.
struct HeadAttnImpl : torch::nn::Module {
    torch::Tensor weight, bias;
    HeadAttnImpl(int64_t in, int64_t heads);
};
TORCH_MODULE(HeadAttn);
// [N, H]: out[:, h] = X[:, hD:(h+1)D] . weight[hD:(h+1)D] + bias[h] (torch ops, autograd)
torch::Tensor head_attn_apply(torch::Tensor X, torch::Tensor weight, torch::Tensor bias);

// The first layer of a multi-head GAT program in input space (include/gala_hip.h
// gala_gat_in_*): the value and gradients of
//   gat_aggregate_ffn_apply(head_attn_apply(v1, attn_l_weight, attn_l_bias), v1,
//                           attn_r_weight, attn_r_bias, li, slope, mode),   v1 = ffn_apply(X, weight, bias)
// with the edges gathering X's rows (fin floats) instead of v1's (H*D).  Used when X needs
// no gradient (the dataset's features), fin < H*D <= 8*32, REF softmax on the undirected
// graph without hub rows; otherwise it runs the three ops themselves (GALA_GAT_INPUT=0: always).
// relu: the program's torch::relu on the layer's output fused (forward store, backward mask).
bool gat_input_layer_eligible(const torch::Tensor &X, const torch::Tensor &W, int64_t li, int64_t heads, int64_t mode);
torch::Tensor gat_input_layer_apply(torch::Tensor X, torch::Tensor weight, torch::Tensor bias,
                                    torch::Tensor attn_l_weight, torch::Tensor attn_l_bias,
                                    torch::Tensor attn_r_weight, torch::Tensor attn_r_bias, int64_t li,
                                    double slope, int64_t mode, bool relu = false);

}  // namespace gala
