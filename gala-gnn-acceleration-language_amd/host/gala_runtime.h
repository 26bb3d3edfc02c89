// gala_runtime.h — host runtime of the programs galac emits (compiler/emit.cpp).
//
// Replaces what the reference's emitted gala.cu pulls from tests/common.h and
// src/utils/* (readSM_npy32 / readDM_npy, getMaskSubgraphs, ord_col_tiling_torch,
// inplace_sample_graph_ab, get_time / calc_mean, printMemoryUsage) and the device-side
// setup of codegen/gala.cu:461-600 (cudaMalloc + cudaMemcpy + from_blob + the
// global_*_graph pushes).  Host preprocessing goes through the C ABI's builders
// (include/gala_hip.h); device graphs are registered in gala::global_slots().
#pragma once

#include <torch/torch.h>

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "gala_torch.h"

namespace gala {
namespace rt {

// Command line of an emitted program:
//   --data DIR      dataset directory (Adj_src.npy, Adj_dst.npy, Feat.npy, Lab.npy,
//                   TnMsk.npy, VlMsk.npy, TsMsk.npy as written by gala_export_npy.py)
//   --synthetic     ignore any dataset directory, generate the dataset's shape
//   --scale S       synthetic: scale vertex and edge counts by S (shape smoke runs)
//   --iters N       override the DSL's iteration count
//   --seed N        weight init / synthetic data seed
//   --dump FILE     write the first forward's inputs, weights and output (parity tests)
//   --quiet         only the reference's result line
//   --device D      gpu (default: cuda:0, libgala_hip.so) or cpu (host cores,
//                   libgala_cpu.so; the reference has no CPU backend, src/codegen/cpu.h)
struct RunArgs {
    std::string data_dir, dump_path, device = "gpu";
    bool synthetic = false, quiet = false;
    double scale = 1.0;
    int64_t iters = -1;
    uint64_t seed = 1;
};
RunArgs parse_args(int argc, char **argv);
torch::Device device(const RunArgs &args);  // --device: where every tensor of the run lives
void sync(const torch::Device &dev);         // device barrier before a timestamp (no-op on CPU)

// A dataset on the host (CPU tensors).
struct Dataset {
    std::string name, source;  // source: the directory read, or "synthetic"
    int64_t n = 0;
    torch::Tensor rowptr, col;  // int32 CSR, rows = src (readSM_npy32), cols ascending
    torch::Tensor feat;         // float32 [n, F]
    torch::Tensor labels;       // int64 [n]
    torch::Tensor train_mask, valid_mask, test_mask;  // bool [n]
    int64_t classes = 0;
};
// `name` is the DSL's load_dataset argument; the directory is --data, else opt_input,
// else Data/<name>/ under the working directory, else a synthetic graph of the
// dataset's published shape (uniform random, symmetric, with self loops; features
// U[-1,1), random labels).  feat_size / label_size (the DSL's feature_size /
// label_size, <= 0 if not given) size the synthetic data and are checked against files.
Dataset load_dataset(const std::string &name, const RunArgs &args, int64_t feat_size,
                     int64_t label_size, const std::string &opt_input = "");

// Graph layout the schedule asks for.
struct GraphPlan {
    bool undirected = true;     // backward slot shares the forward tensors (cuda.h:1253-1257)
    bool weighted = false;      // !set_unweighted: aggregations read value_graph
    int64_t col_tile = 0;       // COL_TILE: columns per segment (0 = untiled)
    int64_t data_sample = 0;    // G.sample(n): inplace_sample_graph_ab(n, 5, 7)
    int subgraph_levels = 0;    // training subgraph: graphs 1..L = mask levels L-1..0
    bool transpose_perm = false;  // register edge permutations for FIXED-mode GAT
};
// Registers graph g as slots 2g (forward) / 2g+1 (backward) of global_slots():
// graph 0 is the whole graph; with subgraph_levels = L, graph 1 + c is the c-th
// aggregation's subgraph (mask level L-1-c).  Returns the number of graphs.
int prepare_graphs(const Dataset &ds, const GraphPlan &plan, torch::Device dev);

// Kernel sampling (aggrFn.sample(n) / .sample(n).dynamic(); common.h:813-833).
void set_kernel_sampling(int64_t nsamples, bool dynamic, uint64_t seed);
void next_forward();  // dynamic sampling: fresh (ra, rb) in [0, 100]
// FULL_OP degrees of a kernel-sampled graph: full({N, 1}, n * segments) (common.h:1342-1374)
torch::Tensor sampled_degrees(int64_t nsamples);
// DEGREES: rows' edge counts of graph 0, summed over its segments (gala.cu:433-440)
torch::Tensor degrees();

// torch::nn::CrossEntropyLoss (mean reduction) as -mean(log_softmax(pred)[i, y_i]): the
// same value and gradient without nll_loss's single-workgroup reduction kernels
torch::Tensor cross_entropy(const torch::Tensor &pred, const torch::Tensor &labels);
double get_time();
double calc_mean(const std::vector<double> &v);
int64_t device_memory_mb(const torch::Device &dev);  // printMemoryUsage (cuda.h:1000-1020):
                                                     // used device memory (CPU: resident MB)

// --dump: named tensors to a flat little-endian file (name, dtype, shape, bytes)
void dump(const std::string &path,
          const std::vector<std::pair<std::string, torch::Tensor>> &tensors);

}  // namespace rt
}  // namespace gala
