// pybind11 module gala._gala_torch: exposes the C++ operator mirror (gala_torch.h) to
// Python so the parity tests exercise the same C++ entry points a generated program calls.
#include <torch/extension.h>

#include "gala_torch.h"

namespace py = pybind11;
using namespace gala;

PYBIND11_MODULE(_gala_torch, m) {
    m.doc() = "C++/libtorch mirror of GALA's emitted operator API over libgala_hip.so";

    m.def("slots_clear", []() { global_slots().clear(); });
    m.def("slots_push",
          [](torch::Tensor off, torch::Tensor cols, std::optional<torch::Tensor> vals,
             std::optional<torch::Tensor> bounds, int segments, bool weighted) {
              return global_slots().push(off, cols, vals ? *vals : torch::Tensor(),
                                         bounds ? *bounds : torch::Tensor(), segments, weighted);
          },
          py::arg("offset_graph"), py::arg("columns_graph"), py::arg("value_graph"),
          py::arg("bounds"), py::arg("segments") = 1, py::arg("weighted") = false);
    m.def("slots_set_value", [](int idx, torch::Tensor v, bool weighted) {
        global_slots().value_graph.at(idx) = v;
        global_slots().weighted.at(idx) = weighted;
    });
    m.def("slots_set_transpose_perm",
          [](int idx, torch::Tensor perm) { global_slots().transpose_perm.at(idx) = perm; });
    m.def("slots_set_sampling", [](int nsamples, int ra, int rb) {
        auto &S = global_slots();
        S.nsamples = nsamples;
        S.ra = ra;
        S.rb = rb;
    });
    m.def("slots_size", []() { return (int)global_slots().offset_graph.size(); });

    // optional tensors: None -> undefined tensor (the reference passes no bounds when untiled)
    auto opt = [](const std::optional<torch::Tensor> &t) { return t ? *t : torch::Tensor(); };
    m.def("aggregate_node_mul_sum_call",
          [opt](torch::Tensor x, torch::Tensor off, torch::Tensor cols, torch::Tensor vals,
                std::optional<torch::Tensor> bounds, int64_t segments, bool weighted,
                int64_t nsamples, int64_t ra, int64_t rb) {
              return aggregate_node_mul_sum_call(x, off, cols, vals, opt(bounds), segments,
                                                 weighted, nsamples, ra, rb);
          },
          py::arg("input_dense"), py::arg("offset_graph"), py::arg("columns_graph"),
          py::arg("value_graph"), py::arg("bounds") = py::none(), py::arg("segments") = 1,
          py::arg("weighted") = false, py::arg("nsamples") = 0, py::arg("ra") = 5,
          py::arg("rb") = 7);
    m.def("aggregate_node_mul_sum_direct_call",
          [opt](torch::Tensor x, torch::Tensor off, torch::Tensor cols, torch::Tensor vals,
                std::optional<torch::Tensor> bounds, int64_t segments, bool weighted) {
              return aggregate_node_mul_sum_direct_call(x, off, cols, vals, opt(bounds), segments,
                                                        weighted);
          },
          py::arg("input_dense"), py::arg("offset_graph"), py::arg("columns_graph"),
          py::arg("value_graph"), py::arg("bounds") = py::none(), py::arg("segments") = 1,
          py::arg("weighted") = false);
    m.def("gather_forward", &gather_forward);
    m.def("node_spmv_backward_of_sddmm_nln", &node_spmv_backward_of_sddmm_nln);
    m.def("node_spmv_backward_of_sddmm_eaggr", &node_spmv_backward_of_sddmm_eaggr);
    m.def("inplace_softmax_sddvv", &inplace_softmax_sddvv);
    m.def("inplace_softmax_sddvv_mult", &inplace_softmax_sddvv_mult);
    m.def("edge_sddvv", &edge_sddvv);
    m.def("edge_sddmm", &edge_sddmm);
    m.def("aggregate_edge_mul", &aggregate_edge_mul);
    m.def("aggregate_edge_mul_dir", &aggregate_edge_mul_dir);
    m.def("row_broadcast", &row_broadcast);
    m.def("degree_norm",
          [opt](torch::Tensor off, std::optional<torch::Tensor> bounds, int64_t segments,
                double power, std::optional<torch::Tensor> cols) {
              return degree_norm(off, opt(bounds), segments, power, opt(cols));
          },
          py::arg("offset_graph"), py::arg("bounds") = py::none(), py::arg("segments") = 1,
          py::arg("power") = -0.5, py::arg("columns_graph") = py::none());
    m.def("gcn_aggregate",
          [opt](torch::Tensor x, torch::Tensor norm, torch::Tensor off, torch::Tensor cols,
                std::optional<torch::Tensor> bounds, int64_t segments) {
              return gcn_aggregate(x, norm, off, cols, opt(bounds), segments);
          },
          py::arg("X"), py::arg("norm"), py::arg("offset_graph"), py::arg("columns_graph"),
          py::arg("bounds") = py::none(), py::arg("segments") = 1);

    m.def("aggregate_node_mul_sum_apply", &aggregate_node_mul_sum_apply);
    m.def("aggregate_node_mul_sum_attn_apply", &aggregate_node_mul_sum_attn_apply);
    m.def("aggregate_edge_sum_apply", &aggregate_edge_sum_apply);
    m.def("non_lnr_op_softmax_apply", &non_lnr_op_softmax_apply);
    m.def("gcn_aggregate_apply",
          [opt](torch::Tensor x, std::optional<torch::Tensor> pre,
                std::optional<torch::Tensor> post, int64_t li) {
              return gcn_aggregate_apply(x, opt(pre), opt(post), li);
          },
          py::arg("X"), py::arg("pre") = py::none(), py::arg("post") = py::none(),
          py::arg("li") = 0);
    m.def("gcn_aggregate_relu_apply",
          [opt](torch::Tensor x, std::optional<torch::Tensor> act, std::optional<torch::Tensor> pre,
                std::optional<torch::Tensor> post, int64_t li) {
              return gcn_aggregate_relu_apply(x, opt(act), opt(pre), opt(post), li);
          },
          py::arg("X"), py::arg("act") = py::none(), py::arg("pre") = py::none(),
          py::arg("post") = py::none(), py::arg("li") = 0);
    m.def("ffn_apply",
          [opt](torch::Tensor x, torch::Tensor w, std::optional<torch::Tensor> b) {
              return ffn_apply(x, w, opt(b));
          },
          py::arg("X"), py::arg("weight"), py::arg("bias") = py::none());
    m.def("head_attn_apply", &head_attn_apply, py::arg("X"), py::arg("weight"), py::arg("bias"));
    m.def("gat_aggregate_apply", &gat_aggregate_apply, py::arg("attn_l"), py::arg("attn_r"),
          py::arg("X"), py::arg("li"), py::arg("slope") = 0.2, py::arg("mode") = 0);
    m.def("gat_aggregate_ffn_apply", &gat_aggregate_ffn_apply, py::arg("attn_l"), py::arg("X"),
          py::arg("attn_r_weight"), py::arg("attn_r_bias"), py::arg("li"), py::arg("slope") = 0.2,
          py::arg("mode") = 0);
    m.def("gat_input_layer_apply",
          [opt](torch::Tensor x, torch::Tensor w, std::optional<torch::Tensor> b, torch::Tensor wl, torch::Tensor bl,
                torch::Tensor wr, torch::Tensor br, int64_t li, double slope, int64_t mode, bool relu) {
              return gat_input_layer_apply(x, w, opt(b), wl, bl, wr, br, li, slope, mode, relu);
          },
          py::arg("X"), py::arg("weight"), py::arg("bias"), py::arg("attn_l_weight"), py::arg("attn_l_bias"),
          py::arg("attn_r_weight"), py::arg("attn_r_bias"), py::arg("li"), py::arg("slope") = 0.2,
          py::arg("mode") = 0, py::arg("relu") = false);
    m.def("gat_input_layer_eligible", &gat_input_layer_eligible);
}
