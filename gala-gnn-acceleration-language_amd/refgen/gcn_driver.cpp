// gcn_driver.cpp -- the reference compiler's driver (tests/gala_inference.cpp:100-190) with
// the HIP code generator (refgen/hip.h), fed a hand-built GCN IR.
//
// The reference's parser is bison/flex (src/frontend/frontend.{y,l}), absent from this image,
// so the IR a GCN program parses into is built here directly, node for node and edge for
// edge as the front-end's actions build it for the GCN layer template
//     deg = G.graphs.degrees(); norm = dsl.fn.pow(deg, p); res = norm * feats;
//     res = aggregate_fn(G.graphs, res); res = dsl.nn.ffn(res, out=hs); res = norm * res;
//     feats = nonln_fn(res)
// (layer operations GET_DEGREES, GET_NORMALIZATION, MULT_NORM_RES, MESSAGE_PASSING_AGGREGATE,
// FEED_FORWARD_NN, MULT_NORM_RES, NON_LINEARITY: frontend.y:463-650 for the ops, 940-1030
// for the layer walk, 1031-1108 for the program).  Then, as gala_inference does, the
// middle-end's operator reordering and sparse rewrites run and the generator writes
// CMakeLists.txt and gala.cu into the output directory.
//
// Compiled against the reference's own headers where they lie (-I <reference>,
// -I <reference>/src/codegen); nothing of the reference is copied.
//
// usage: gcn_driver OUT_DIR/ DATASET FEAT LABELS HIDDEN ITERS [COARSEN]
#include <cstdlib>
#include <iostream>
#include <string>
#include <vector>

#include "hip.h"
#include "src/middle-end/middle-end.h"

std::vector<CIRNode *> GALAFEContext::program;
std::vector<RelationEdge *> GALAFEContext::dependencies;
std::vector<RelationEdge *> GALAFEContext::associations;
std::vector<TransformEdge *> GALAFEContext::transforms;
bool GALAFEContext::operator_reordering = true;   // gala_inference's defaults
bool GALAFEContext::sparse_rewrites = true;
bool GALAFEContext::train_code_motion = true;
bool GALAFEContext::training_subgraph = true;
bool GALAFEContext::print_accuracy = false;
bool GALAFEContext::print_memory = false;
bool GALAFEContext::use_long = false;
std::string GALAFEContext::opt_input = "";

namespace {

struct GcnSpec {
    std::string dataset;
    int feat = 0, labels = 0, hidden = 0, iterations = 1, coarsen = 0;
    float power = -0.5f;
    int layers = 2;
    bool relu(int l) const { return l + 1 < layers; }  // nonln_fn on every layer but the output
};

DataNode *tensorNode(const std::string &name, int rows, int cols, DataFormat fmt = RM_DTYPE) {
    auto *info = new DataInfo(fmt, false, false);
    info->setDims(rows, cols);
    return new DataNode(name, INT32, INT32, F32, new DataLevel(info, true));
}

void depend(DataNode *from, RelationDim r1, DataNode *to, RelationDim r2) {
    GALAFEContext::dependencies.push_back(new RelationEdge(from, r1, to, r2));
}
void associate(DataNode *a, RelationDim r1, DataNode *b, RelationDim r2) {
    GALAFEContext::associations.push_back(new RelationEdge(a, r1, b, r2));
}

ForwardNode *op(TrainingLoopNode *loop, OpType t, ComputeOp o, std::vector<DataNode *> in, DataNode *out) {
    auto *n = new ForwardNode(t, o);
    for (DataNode *d : in) n->addInputData(d);
    if (out) n->addOutputData(out);
    loop->addLoopNode(n);
    return n;
}

// The program the front-end builds for a GCN model of `layers` layers (hidden width
// `hidden`, the last layer's width the label count).
void buildGcn(const GcnSpec &s) {
    auto *load = new ForwardNode(POINTWISE, LOAD_OP);
    load->addParam(s.dataset);
    auto *ginfo = new DataInfo(CSR_STYPE, false, true);
    ginfo->setDims(0, 0);
    DataNode *graph = new DataNode("adj0", INT32, INT32, F32, new DataLevel(ginfo, true));
    DataNode *feat = tensorNode("t_iden", -1, -2);
    associate(graph, ALL_RELATION, feat, ROWS_RELATION);
    load->addOutputData(feat);
    load->addOutputData(graph);
    GALAFEContext::program.push_back(load);
    // no data transformation: the schedule lands on the loaded graph (undirected, unweighted)
    ginfo->setWeighted(false);
    ginfo->setSparse(false);
    ginfo->setIndex(0);
    feat->getDataInfo()->setDims(-1, s.feat);

    auto *loop = new TrainingLoopNode(s.iterations, CROSS_ENTROPY, ADAM, 1);
    DataNode *norm = nullptr, *prev = feat;
    for (int l = 0; l < s.layers; ++l) {
        const bool last = l + 1 == s.layers;
        const int width = last ? s.labels : s.hidden;
        if (l == 0) {  // GET_DEGREES: ones, then the direct (no-autograd) aggregation of them
            DataNode *ones = tensorNode("ones", -1, 1);
            op(loop, POINTWISE, ONES_OP, {}, ones);
            associate(graph, ALL_RELATION, ones, ROWS_RELATION);
            DataNode *deg = tensorNode("degrees", -1, 1);
            ForwardNode *d = op(loop, AGGREGATE_NODE, AGGREGATE_MUL_SUM_DIRECT, {ones, graph}, deg);
            if (s.coarsen) d->addOpt(COARSE_COPT, (float)s.coarsen);
            depend(ones, ALL_RELATION, deg, ALL_RELATION);
            depend(graph, ALL_RELATION, deg, ROWS_RELATION);
            // GET_NORMALIZATION: norm = deg ^ power
            norm = tensorNode("norm", -1, 1);
            ForwardNode *p = op(loop, POINTWISE, POWER_OP, {deg}, norm);
            p->addParam(std::to_string(s.power));
            depend(deg, ALL_RELATION, norm, ALL_RELATION);
        }
        // MULT_NORM_RES: res = norm * (features | the previous layer's output)
        DataNode *scaled = tensorNode("res", -1, l == 0 ? s.feat : s.hidden);
        op(loop, UPDATE_NODE, ROW_BROADCAST_OP, {norm, prev}, scaled);
        depend(norm, ALL_RELATION, scaled, ROWS_RELATION);
        depend(prev, ALL_RELATION, scaled, ALL_RELATION);
        associate(norm, ALL_RELATION, prev, ROWS_RELATION);
        // MESSAGE_PASSING_AGGREGATE
        DataNode *aggr = tensorNode("res", -1, l == 0 ? s.feat : s.hidden);
        ForwardNode *a = op(loop, AGGREGATE_NODE, AGGREGATE_MUL_SUM_OP, {scaled, graph}, aggr);
        if (s.coarsen) a->addOpt(COARSE_COPT, (float)s.coarsen);
        depend(scaled, ALL_RELATION, aggr, ALL_RELATION);
        depend(graph, ALL_RELATION, aggr, ALL_RELATION);
        // FEED_FORWARD_NN: weight<l+1> [in, width]
        DataNode *w = tensorNode("weight" + std::to_string(l + 1), l == 0 ? s.feat : s.hidden, width);
        DataNode *ffn = tensorNode("res", -1, width);
        op(loop, UPDATE_NODE, FFN_OP, {aggr, w}, ffn);
        depend(aggr, ALL_RELATION, ffn, ALL_RELATION);
        depend(w, COLS_RELATION, ffn, ROWS_RELATION);
        associate(aggr, ROWS_RELATION, w, COLS_RELATION);
        // MULT_NORM_RES
        DataNode *post = tensorNode("res", -1, width);
        op(loop, UPDATE_NODE, ROW_BROADCAST_OP, {norm, ffn}, post);
        depend(norm, ALL_RELATION, post, ROWS_RELATION);
        depend(ffn, ALL_RELATION, post, ALL_RELATION);
        associate(norm, ALL_RELATION, ffn, ROWS_RELATION);
        prev = post;
        // NON_LINEARITY
        if (s.relu(l)) {
            DataNode *r = tensorNode("res", -1, width);
            op(loop, POINTWISE, NON_LNR_OP_RELU, {prev}, r);
            depend(prev, ALL_RELATION, r, ALL_RELATION);
            prev = r;
        }
    }
    GALAFEContext::program.push_back(loop);
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 7) {
        std::cerr << "usage: gcn_driver OUT_DIR/ DATASET FEAT LABELS HIDDEN ITERS [COARSEN]\n";
        return 2;
    }
    std::string out = argv[1];
    GcnSpec s;
    s.dataset = argv[2];
    s.feat = std::atoi(argv[3]);
    s.labels = std::atoi(argv[4]);
    s.hidden = std::atoi(argv[5]);
    s.iterations = std::atoi(argv[6]);
    s.coarsen = argc > 7 ? std::atoi(argv[7]) : 0;
    buildGcn(s);
    auto *ctx = new GALAContext(GPU_DEVICE, SINGLE_NODE_SINGLE);
    auto gen = HIPGenerator(ctx, out);
    if (GALAFEContext::operator_reordering)
        GALATransformations::complexityOperatorReordering(GALAFEContext::program, GALAFEContext::dependencies,
                                                          GALAFEContext::associations, GALAFEContext::transforms);
    if (GALAFEContext::sparse_rewrites)
        GALATransformations::sparsityAwareRewrites(GALAFEContext::program, GALAFEContext::dependencies,
                                                   GALAFEContext::associations, GALAFEContext::transforms);
    gen.writeCode(GALAFEContext::program, GALAFEContext::dependencies, GALAFEContext::associations,
                  GALAFEContext::transforms);
    std::cout << "wrote " << out << "gala.cu and " << out << "CMakeLists.txt" << std::endl;
    return 0;
}
