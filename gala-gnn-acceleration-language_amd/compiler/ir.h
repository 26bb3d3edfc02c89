// ir.h — galac's intermediate representation of a GALA program.
//
// The reference lowers a DSL program into CIR: a LOAD node plus a TrainingLoopNode
// holding ComputeNodes (src/ir/compute.h, built by frontend.y:440-1060 generate_ir /
// addLayer).  galac keeps the same op vocabulary (ComputeOp names in comments) but as an
// SSA dataflow list: every node writes one new value, so the middle-end passes
// (passes.cpp) are rewrites over use-def chains instead of name juggling.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "ast.h"

namespace galac {

enum class Op {
    Input,          // t_iden: the dataset's node features                (LOAD_OP)
    Degrees,        // row edge counts of graph 0 [N,1]                   (DEGREES_OP / AGGREGATE_MUL_SUM_DIRECT)
    SampledDegrees, // kernel-sampled degrees: full(n * segments)         (FULL_OP)
    Power,          // x^p                                                (POWER_OP)
    RowBroadcast,   // vec[N,1] * x[N,F]                                  (ROW_BROADCAST_OP)
    Aggregate,      // A x (graph `graph`, edge weights from in[1] if any) (AGGREGATE_MUL_SUM_OP)
    Ffn,            // Linear(in, out) with bias                          (FFN_OP / FFN_OP_EDGE / FFN_OP_SELF)
    Relu,           //                                                    (NON_LNR_OP_RELU)
    EdgeAdd,        // s_e = a[row] + b[col]                              (AGGREGATE_EDGE_SUM_OP)
    LeakyRelu,      // on edge values, slope param                       (NON_LNR_OP_LEAKY_RELU)
    Softmax,        // per-row edge softmax                               (NON_LNR_OP_SOFTMAX)
    ScaleEps,       // (1 + eps) x, eps a learned scalar                  (SCALAR_ADD_EPS_MULTIPLY_OP)
    Add,            // a + b                                              (ADD_OP)
    // produced by the middle-end
    EdgeMul,        // w_e = a[row] * b[col] (sparse rewrite)             (AGGREGATE_EDGE_MUL_OP)
    GcnAggregate,   // post * A (pre * x), fused ROW_BROADCAST/AGGREGATE chain; param 1:
                    // x = relu(act * in[0]) first (in[3] = act | -1), the ReLU prologue
    GatAggregate,   // softmax(lrelu(aL[row] + aR[col])) weighted A x, fused
};
const char *op_name(Op op);

enum class Kind { Node, NodeVec, Edge, Scalar };

struct Value {
    std::string name;  // readable name for dumps / generated code
    Kind kind = Kind::Node;
    int64_t width = 0;      // feature columns (Node), 1 (NodeVec)
    bool invariant = false; // independent of the weights (graph / input-feature data)
};

struct Node {
    Op op;
    std::vector<int> in;    // value ids; Aggregate: {x[, weights]}; GcnAggregate: {x, pre|-1, post|-1[, act|-1]}
    int out = -1;
    double param = 0;       // Power exponent, LeakyRelu slope, ScaleEps initial eps
    int weight = -1;        // Ffn / ScaleEps: index into Module::weights
    int graph = 0;          // Aggregate-like: graph index (slots 2g / 2g+1)
    int layer = -1;         // model layer that produced the node (-1: program level)
    bool hoisted = false;   // computed once before the training loop (code motion)
    bool dead = false;
};

struct Weight {
    std::string name;       // fc<k> / sfc<k> / efc<k> / eps<k> as in gala.cu
    enum Type { Linear, Eps } type = Linear;
    int64_t in = 0, out = 0;
    double init = 0;        // Eps initial value
    int64_t heads = 1;      // > 1: a multi-head attention vector (galac gat_heads(H)): weight
                            // [1, in] read per head slice, bias [heads]; out = 1 per head
};

// Schedule and program-level settings (ModelConfig, ir/frontend_metadata.h:44-140, and
// GALAFEContext flags, frontend/context.h).
struct Schedule {
    std::string dataset;
    std::string opt_input;
    bool undirected = true;        // UNDIRECTED (default true: frontend.y + gala_inference)
    bool unweighted = false;       // UNWEIGHTED
    bool sparse = false;           // is_sparser: SPARSE (gates the sparse rewrite)
    int64_t feat_size = -2;        // FEAT_SIZE (-2: from the data)
    int64_t label_size = -3;       // LABEL_SIZE (-3: from the data)
    int64_t col_tile = 0;          // COL_TILE
    int64_t data_sample = 0;       // G.sample(n): SAMP
    int64_t coarsen = 0;           // COARSE (CUDA launch geometry; recorded, no effect)
    int64_t kernel_sample = 0;     // aggrFn.sample(n): SAMP_CPT
    bool dynamic_sample = false;   // .dynamic(): SAMP_DYN_CPT
    bool print_accuracy = false, print_memory = false;
    bool operator_reordering = true, sparse_rewrites = true, training_subgraph = true,
         train_code_motion = true;
    int64_t iterations = 0, validation_step = 0;
    int gat_mode = 0;              // 0 = reference gradients (GALA_SOFTMAX_REF), 1 = fixed
    int64_t gat_heads = 1;         // galac extension gat_heads(H): attention layers but the
                                   // last run H heads of `hs` features each
};

struct Module {
    std::string source;
    Schedule sched;
    std::vector<Value> values;
    std::vector<Node> nodes;       // program order
    std::vector<Weight> weights;
    int output = -1;               // the model's prediction
    int num_layers = 0;
    int num_graphs = 1;            // graph 0 = whole graph (+ training subgraphs)
    std::vector<std::string> notes;  // lowering / pass decisions, printed by galac

    int add_value(const std::string &name, Kind k, int64_t width, bool invariant);
    int add_node(Node n);
    std::vector<int> uses(int value) const;  // live nodes reading `value`
    int producer(int value) const;           // live node writing `value` (-1: none)
    std::string dump() const;
    std::string to_json() const;  // machine-readable IR (tests/_ir_ref.py executes it)
};

// Parse-tree -> IR (lower.cpp).  Throws DslError on programs it cannot give meaning to.
Module lower(const Program &prog);
// Middle-end (passes.cpp), in the order gala_train.cpp:124-146 runs them, followed by
// the MI355X fusions.
void run_passes(Module &m, bool fuse = true);
// HIP emitter (emit.cpp): a C++ program over gala_torch.h / gala_runtime.h.
std::string emit_program(const Module &m);
std::string emit_makefile(const Module &m, const std::string &pkg_dir);

}  // namespace galac
