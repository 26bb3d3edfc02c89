// ir_driver.cpp -- the reference compiler's driver (tests/gala_inference.cpp:100-190) with
// the HIP code generator (refgen/hip.h), fed a hand-built IR of a GCN, GAT, GIN or
// GraphSAGE program (the four model families of tests/GALA-DSL).
//
// The reference's parser is bison/flex (src/frontend/frontend.{y,l}), absent from this image,
// so the IR a program parses into is built here directly, node for node and edge for edge as
// the front-end's actions build it:
//   gcn  the GCN layer template
//            deg = G.graphs.degrees(); norm = dsl.fn.pow(deg, p); res = norm * feats;
//            res = aggregate_fn(G.graphs, res); res = dsl.nn.ffn(res, out=hs);
//            res = norm * res; feats = nonln_fn(res)
//        (layer operations GET_DEGREES, GET_NORMALIZATION, MULT_NORM_RES,
//        MESSAGE_PASSING_AGGREGATE, FEED_FORWARD_NN, MULT_NORM_RES, NON_LINEARITY);
//   gat  the GAT layer template of tests/GALA-DSL/gat/*
//            res = dsl.nn.ffn(feats, out=hs); attnL = dsl.nn.ffn(res, out=1);
//            attnR = dsl.nn.ffn(res, out=1); attn = edge_fn(G, attnL, attnR);
//            G.edges.vals = dsl.fn.softmax(G, attn); res = aggregate_fn(G.graphs, res);
//            feats = nonln_fn(res)
//        (FEED_FORWARD_NN, ATTEN_L -- which also adds the right attention Linear and the
//        edge sum --, ATTN (the LeakyReLU), SOFTMAX_OP, MESSAGE_PASSING_AGGREGATE,
//        NON_LINEARITY), over the column-tiled graph `graph_tile` its schedule's col_tile
//        asks for (generate_ir's transformed graph).
// frontend.y:471-802 for the ops, 940-1030 for the layer walk, 1031-1108 for the program.
// Then, as gala_inference does, the middle-end's operator reordering and sparse rewrites run
// (with GALA_REFGEN_CODE_MOTION set, also gala_train's training-invariant code motion) and the
// generator writes CMakeLists.txt and gala.cu into the output directory.
//
// Compiled against the reference's own headers where they lie (-I <reference>,
// -I <reference>/src/codegen); nothing of the reference is copied.
//
// usage: ir_driver OUT_DIR/ gcn|gcn3|gat|gin|sage DATASET FEAT LABELS HIDDEN ITERS
//                  [COARSEN [COL_TILE [NSAMP [DATA_SAMPLE]]]]
// (NSAMP: aggrFn.sample(NSAMP), the kernel-sampled GCN of tests/GALA-DSL/ablations/sampling/kernel;
// DATA_SAMPLE: G.sample(n), the data-sampled GCN of tests/GALA-DSL/ablations/sampling/data)
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

struct Spec {
    std::string model, dataset;
    int feat = 0, labels = 0, hidden = 0, iterations = 1, coarsen = 0, col_tile = 0;
    int nsamp = 0;        // aggrFn.sample(n): kernel sampling (compute transformation SAMP_CPT)
    int data_samp = 0;    // G.sample(n): data sampling (graph transformation SAMP, SAMPLE_DOPT)
    bool sparse = false;  // G.is_sparser(true)
    float power = -0.5f;
    int layers = 2;
    int validation = 1;   // m1.train(validation_step=): the loop's stepValid (frontend.y:1089)
    bool relu(int l) const { return l + 1 < layers; }  // nonln_fn on every layer but the output
    int width(int l) const { return l + 1 < layers ? hidden : labels; }
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

ForwardNode *op(TrainingLoopNode *loop, OpType nt, ComputeOp o, std::vector<DataNode *> in, DataNode *out) {
    auto *n = new ForwardNode(nt, o);
    for (DataNode *d : in) n->addInputData(d);
    if (out) n->addOutputData(out);
    loop->addLoopNode(n);
    return n;
}

// generate_ir's LOAD node (frontend.y:1035-1050) and the graph the layers run on: the loaded
// one with the schedule's flags (no data transformation), or the transformed `graph_tile`
// (col_tile: frontend.y:1053-1083)
DataNode *loadProgram(const Spec &s, DataNode *&feat) {
    auto *load = new ForwardNode(POINTWISE, LOAD_OP);
    load->addParam(s.dataset);
    auto *ginfo = new DataInfo(CSR_STYPE, false, true);
    ginfo->setDims(0, 0);
    DataNode *graph = new DataNode("adj0", INT32, INT32, F32, new DataLevel(ginfo, true));
    feat = tensorNode("t_iden", -1, -2);
    associate(graph, ALL_RELATION, feat, ROWS_RELATION);
    load->addOutputData(feat);
    load->addOutputData(graph);
    GALAFEContext::program.push_back(load);
    feat->getDataInfo()->setDims(-1, s.feat);
    if (!s.col_tile) {  // undirected, unweighted, not sparse: the loaded graph itself
        ginfo->setWeighted(false);
        ginfo->setSparse(false);
        ginfo->setIndex(0);
        return graph;
    }
    // undirected, unweighted, the schedule's is_sparser
    auto *tinfo = new DataInfo(CSR_STYPE, false, false);
    tinfo->setSparse(s.sparse);
    if (s.data_samp) tinfo->addOpt(SAMPLE_DOPT, std::to_string(s.data_samp));
    tinfo->addOpt(COL_TILE_DOPT, std::to_string(s.col_tile));
    auto *tile = new DataNode("graph_tile", graph->getIType(), graph->getNType(), graph->getVType(),
                              new DataLevel(new DataLevel(tinfo, false), true));
    associate(tile, ALL_RELATION, feat, ROWS_RELATION);
    auto *edge = new TransformEdge(graph, tile);
    if (s.data_samp) {  // the sampled rows first, then the column tiles of them
        auto *samp = new TransformData(SAMPLE_DOPT);
        samp->addParam(std::to_string(s.data_samp));
        edge->addTransformation(samp);
    }
    auto *tr = new TransformData(COL_TILE_DOPT);
    tr->addParam(std::to_string(s.col_tile));
    edge->addTransformation(tr);
    GALAFEContext::transforms.push_back(edge);
    return tile;
}

// addFFN_CIR (frontend.y:590-635): weight<l+1> [in, width]
DataNode *ffnNode(TrainingLoopNode *loop, const Spec &s, int l, DataNode *in) {
    DataNode *w = tensorNode("weight" + std::to_string(l + 1), l == 0 ? s.feat : s.hidden, s.width(l));
    DataNode *out = tensorNode("res", -1, s.width(l));
    op(loop, UPDATE_NODE, FFN_OP, {in, w}, out);
    depend(in, ALL_RELATION, out, ALL_RELATION);
    depend(w, COLS_RELATION, out, ROWS_RELATION);
    associate(in, ROWS_RELATION, w, COLS_RELATION);
    return out;
}

// NON_LINEARITY (addReLU_CIR, frontend.y:636-648)
DataNode *reluNode(TrainingLoopNode *loop, int width, DataNode *in) {
    DataNode *r = tensorNode("res", -1, width);
    op(loop, POINTWISE, NON_LNR_OP_RELU, {in}, r);
    depend(in, ALL_RELATION, r, ALL_RELATION);
    return r;
}

// The program the front-end builds for a GCN model of `layers` layers (hidden width
// `hidden`, the last layer's width the label count).
void buildGcn(const Spec &s) {
    DataNode *feat = nullptr;
    DataNode *graph = loadProgram(s, feat);
    auto *loop = new TrainingLoopNode(s.iterations, CROSS_ENTROPY, ADAM, s.validation);
    DataNode *norm = nullptr, *prev = feat;
    for (int l = 0; l < s.layers; ++l) {
        if (l == 0 && s.nsamp) {  // GET_DEGREES of a kernel-sampled program: nsamp per row
            DataNode *deg = tensorNode("degrees", -1, 1);
            ForwardNode *d = op(loop, UPDATE_NODE, FULL_OP, {graph}, deg);
            d->addParam(std::to_string((float)s.nsamp));
            depend(graph, ALL_RELATION, deg, ROWS_RELATION);
            norm = tensorNode("norm", -1, 1);
            ForwardNode *p = op(loop, POINTWISE, POWER_OP, {deg}, norm);
            p->addParam(std::to_string(s.power));
            depend(deg, ALL_RELATION, norm, ALL_RELATION);
        } else if (l == 0) {  // GET_DEGREES: ones, then the direct (no-autograd) aggregation of them
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
        if (s.nsamp) a->addOpt(SAMPLE_COPT, (float)s.nsamp);
        depend(scaled, ALL_RELATION, aggr, ALL_RELATION);
        depend(graph, ALL_RELATION, aggr, ALL_RELATION);
        // FEED_FORWARD_NN
        DataNode *ffn = ffnNode(loop, s, l, aggr);
        // MULT_NORM_RES
        DataNode *post = tensorNode("res", -1, s.width(l));
        op(loop, UPDATE_NODE, ROW_BROADCAST_OP, {norm, ffn}, post);
        depend(norm, ALL_RELATION, post, ROWS_RELATION);
        depend(ffn, ALL_RELATION, post, ALL_RELATION);
        associate(norm, ALL_RELATION, ffn, ROWS_RELATION);
        prev = s.relu(l) ? reluNode(loop, s.width(l), post) : post;
    }
    GALAFEContext::program.push_back(loop);
}

// addAttentionWeight_L / _R (frontend.y:649-736): an FFN_OP_EDGE of the layer's FFN output
// (the generator makes it Linear(width, 1), common.h:1248-1260)
DataNode *attentionNode(TrainingLoopNode *loop, const Spec &s, int l, const char *side, DataNode *res) {
    auto *winfo = new DataInfo(CM_DTYPE);
    winfo->setDims(l == 0 ? s.feat : s.hidden, s.width(l));
    DataNode *w = new DataNode(std::string("atten") + side + "Weight" + std::to_string(l + 1), INT32, INT32, F32,
                               new DataLevel(winfo, true));
    const std::string name = std::string("atten") + side + (l ? "_" + std::to_string(l + 1) : "");
    DataNode *out = tensorNode(name, -1, s.width(l));
    op(loop, UPDATE_NODE, FFN_OP_EDGE, {res, w}, out);
    depend(res, ALL_RELATION, out, ALL_RELATION);
    depend(w, COLS_RELATION, out, ROWS_RELATION);
    associate(res, ROWS_RELATION, w, COLS_RELATION);
    return out;
}

// an edge-valued result over the graph ("attn"): CSR, undirected, weighted
DataNode *edgeNode(const Spec &s, bool tiled_derived) {
    auto *info = new DataInfo(CSR_STYPE, false, true);
    if (tiled_derived) {
        info->addOpt(COL_TILE_DOPT, std::to_string(s.col_tile));
        info->setIndex(0);
        info->setDerived(true);
    }
    return new DataNode("attn", INT32, INT32, F32, new DataLevel(info, true));
}

// The program the front-end builds for the GAT layer template (tests/GALA-DSL/gat/*).
void buildGat(const Spec &s) {
    DataNode *feat = nullptr;
    DataNode *graph = loadProgram(s, feat);
    auto *loop = new TrainingLoopNode(s.iterations, CROSS_ENTROPY, ADAM, s.validation);
    DataNode *prev = feat;
    for (int l = 0; l < s.layers; ++l) {
        // FEED_FORWARD_NN
        DataNode *res = ffnNode(loop, s, l, prev);
        // ATTEN_L: both attention Linears, then the edge sum (addAttn, frontend.y:737-767)
        DataNode *aL = attentionNode(loop, s, l, "L", res);
        DataNode *aR = attentionNode(loop, s, l, "R", res);
        DataNode *attn = edgeNode(s, true);
        op(loop, AGGREGATE_EDGE, AGGREGATE_EDGE_SUM_OP, {aL, aR, graph}, attn);
        depend(aL, ALL_RELATION, attn, ROWS_RELATION);
        depend(aR, ALL_RELATION, attn, COLS_RELATION);
        depend(graph, ALL_RELATION, attn, ALL_RELATION);
        associate(graph, ROWS_RELATION, aL, ALL_RELATION);
        associate(graph, COLS_RELATION, aR, ALL_RELATION);
        // ATTN: LeakyReLU(0.2) of the edge values (addLeakyReLU, frontend.y:787-802)
        DataNode *lrelu = edgeNode(s, false);
        ForwardNode *lr = op(loop, UPDATE_EDGE, NON_LNR_OP_LEAKY_RELU, {attn}, lrelu);
        lr->addParam("0.2");
        depend(attn, ALL_RELATION, lrelu, ALL_RELATION);
        // SOFTMAX_OP (addSoftmax_CIR, frontend.y:768-786, with its fixed tile option on the input)
        DataNode *alpha = edgeNode(s, true);
        lrelu->getDataInfo()->addOpt(COL_TILE_DOPT, "300000");
        op(loop, UPDATE_EDGE, NON_LNR_OP_SOFTMAX, {lrelu}, alpha);
        depend(lrelu, ALL_RELATION, alpha, ALL_RELATION);
        // MESSAGE_PASSING_AGGREGATE after the softmax: the FFN output over the edge values
        DataNode *aggr = tensorNode("res", -1, l == 0 ? s.feat : s.hidden);
        ForwardNode *a = op(loop, AGGREGATE_NODE, AGGREGATE_MUL_SUM_OP, {res, alpha}, aggr);
        if (s.coarsen) a->addOpt(COARSE_COPT, (float)s.coarsen);
        depend(res, ALL_RELATION, aggr, ALL_RELATION);
        depend(alpha, ALL_RELATION, aggr, ALL_RELATION);
        prev = s.relu(l) ? reluNode(loop, s.width(l), aggr) : aggr;
    }
    GALAFEContext::program.push_back(loop);
}

// The program the front-end builds for the GIN layer template of tests/GALA-DSL/gin/*
//     res_n = aggregate_fn(G.graphs, feats); res = dsl.nn.scalar(1) * feats;
//     res = res + res_n; res = dsl.nn.ffn(res, out=hs); feats = nonln_fn(res)
// (MESSAGE_PASSING_AGGREGATE, MULT_SCALAR_FEATS, ADD_SCALAR_AGGR, FEED_FORWARD_NN,
// NON_LINEARITY: frontend.y:562-589, 803-835, 965-1019).
void buildGin(const Spec &s) {
    DataNode *feat = nullptr;
    DataNode *graph = loadProgram(s, feat);
    auto *loop = new TrainingLoopNode(s.iterations, CROSS_ENTROPY, ADAM, s.validation);
    DataNode *prev = feat;
    for (int l = 0; l < s.layers; ++l) {
        const int in = l == 0 ? s.feat : s.hidden;
        // MESSAGE_PASSING_AGGREGATE before MULT_SCALAR_FEATS: the output is "res_n"
        DataNode *aggr = tensorNode("res_n", -1, in);
        ForwardNode *a = op(loop, AGGREGATE_NODE, AGGREGATE_MUL_SUM_OP, {prev, graph}, aggr);
        if (s.coarsen) a->addOpt(COARSE_COPT, (float)s.coarsen);
        depend(prev, ALL_RELATION, aggr, ALL_RELATION);
        depend(graph, ALL_RELATION, aggr, ALL_RELATION);
        // MULT_SCALAR_FEATS: (1 + eps) * (the features | the previous layer's ReLU output)
        DataNode *scaled = tensorNode("res", -1, in);
        ForwardNode *e = op(loop, POINTWISE, SCALAR_ADD_EPS_MULTIPLY_OP, {prev}, scaled);
        e->addParam("1");
        depend(prev, ALL_RELATION, scaled, ALL_RELATION);
        // ADD_SCALAR_AGGR
        DataNode *sum = tensorNode("res", -1, in);
        op(loop, UPDATE_NODE, ADD_OP, {scaled, aggr}, sum);
        depend(scaled, ALL_RELATION, sum, ALL_RELATION);
        depend(aggr, ALL_RELATION, sum, ALL_RELATION);
        associate(scaled, ALL_RELATION, aggr, ALL_RELATION);
        DataNode *ffn = ffnNode(loop, s, l, sum);
        prev = s.relu(l) ? reluNode(loop, s.width(l), ffn) : ffn;
    }
    GALAFEContext::program.push_back(loop);
}

// The program the front-end builds for the GraphSAGE-mean layer template of
// tests/GALA-DSL/sage/*
//     res_n = aggregate_fn(G.graphs, feats);            (fn = dsl.fn.mul_mean)
//     res = dsl.nn.ffn(res_n, out=hs) + dsl.nn.ffn(res, out=hs); feats = nonln_fn(res)
// (the SAGE_OPS statement makes the layer GET_DEGREES, GET_NORMALIZATION (power -1),
// MESSAGE_PASSING_AGGREGATE, MULT_NORM_RES, ADD_TWO_FFN, NON_LINEARITY: frontend.y:161-168,
// 471-561, 836-928, 949-1022).
void buildSage(const Spec &s) {
    DataNode *feat = nullptr;
    DataNode *graph = loadProgram(s, feat);
    auto *loop = new TrainingLoopNode(s.iterations, CROSS_ENTROPY, ADAM, s.validation);
    DataNode *norm = nullptr, *prev = feat;
    for (int l = 0; l < s.layers; ++l) {
        const int in = l == 0 ? s.feat : s.hidden;
        if (l == 0) {  // GET_DEGREES, GET_NORMALIZATION (the mean: deg ^ -1)
            DataNode *ones = tensorNode("ones", -1, 1);
            op(loop, POINTWISE, ONES_OP, {}, ones);
            associate(graph, ALL_RELATION, ones, ROWS_RELATION);
            DataNode *deg = tensorNode("degrees", -1, 1);
            ForwardNode *d = op(loop, AGGREGATE_NODE, AGGREGATE_MUL_SUM_DIRECT, {ones, graph}, deg);
            if (s.coarsen) d->addOpt(COARSE_COPT, (float)s.coarsen);
            depend(ones, ALL_RELATION, deg, ALL_RELATION);
            depend(graph, ALL_RELATION, deg, ROWS_RELATION);
            norm = tensorNode("norm", -1, 1);
            ForwardNode *p = op(loop, POINTWISE, POWER_OP, {deg}, norm);
            p->addParam(std::to_string(-1.0f));
            depend(deg, ALL_RELATION, norm, ALL_RELATION);
        }
        // MESSAGE_PASSING_AGGREGATE before MULT_NORM_RES: "res_n"
        DataNode *aggr = tensorNode("res_n", -1, in);
        ForwardNode *a = op(loop, AGGREGATE_NODE, AGGREGATE_MUL_SUM_OP, {prev, graph}, aggr);
        if (s.coarsen) a->addOpt(COARSE_COPT, (float)s.coarsen);
        depend(prev, ALL_RELATION, aggr, ALL_RELATION);
        depend(graph, ALL_RELATION, aggr, ALL_RELATION);
        // MULT_NORM_RES after the aggregation: res_n = norm * res_n
        DataNode *mean = tensorNode("res_n", -1, s.hidden);
        op(loop, UPDATE_NODE, ROW_BROADCAST_OP, {norm, aggr}, mean);
        depend(norm, ALL_RELATION, mean, ROWS_RELATION);
        depend(aggr, ALL_RELATION, mean, ALL_RELATION);
        associate(norm, ALL_RELATION, aggr, ROWS_RELATION);
        // ADD_TWO_FFN: res_n = W1(res_n) (FFN_OP), res = W2(res) (FFN_OP_SELF), res = res_n + res
        auto weight = [&](const char *name) {
            auto *info = new DataInfo(CM_DTYPE);
            info->setDims(in, s.width(l));
            return new DataNode(name, INT32, INT32, F32, new DataLevel(info, true));
        };
        DataNode *w1 = weight("weight1"), *w2 = weight("weight2");
        DataNode *nbr = tensorNode("res_n", -1, s.width(l));
        op(loop, UPDATE_NODE, FFN_OP, {mean, w1}, nbr);
        depend(mean, ALL_RELATION, nbr, ALL_RELATION);
        depend(w1, COLS_RELATION, nbr, ROWS_RELATION);
        associate(mean, ROWS_RELATION, w1, COLS_RELATION);
        DataNode *self = tensorNode("res", -1, s.width(l));
        op(loop, UPDATE_NODE, FFN_OP_SELF, {mean, w2}, self);
        depend(feat, ALL_RELATION, self, ALL_RELATION);
        depend(w2, COLS_RELATION, self, ROWS_RELATION);
        associate(mean, ROWS_RELATION, w2, COLS_RELATION);
        DataNode *sum = tensorNode("res", -1, s.width(l));
        op(loop, UPDATE_NODE, ADD_OP, {nbr, self}, sum);
        depend(nbr, ALL_RELATION, sum, ALL_RELATION);
        depend(self, ALL_RELATION, sum, ALL_RELATION);
        associate(nbr, ALL_RELATION, self, ALL_RELATION);
        prev = s.relu(l) ? reluNode(loop, s.width(l), sum) : sum;
    }
    GALAFEContext::program.push_back(loop);
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 8) {
        std::cerr << "usage: ir_driver OUT_DIR/ gcn|gcn3|gat|gin|sage DATASET FEAT LABELS HIDDEN ITERS "
                     "[COARSEN [COL_TILE [NSAMP [DATA_SAMPLE]]]]\n";
        return 2;
    }
    std::string out = argv[1];
    Spec s;
    s.model = argv[2];
    s.dataset = argv[3];
    s.feat = std::atoi(argv[4]);
    s.labels = std::atoi(argv[5]);
    s.hidden = std::atoi(argv[6]);
    s.iterations = std::atoi(argv[7]);
    s.coarsen = argc > 8 ? std::atoi(argv[8]) : 0;
    s.col_tile = argc > 9 ? std::atoi(argv[9]) : 0;
    s.nsamp = argc > 10 ? std::atoi(argv[10]) : 0;
    s.data_samp = argc > 11 ? std::atoi(argv[11]) : 0;
    if (s.data_samp && !s.col_tile) {  // generate_ir makes the transformed graph only with a data transformation
        std::cerr << "data sampling needs COL_TILE (the reference's transformed graph)\n";
        return 2;
    }
    s.sparse = s.model == "gat";  // the tests/GALA-DSL/gat schedule's is_sparser(true)
    // GALA_REFGEN_TRAIN: gala_train's whole pass set (tests/gala_train.cpp:124-146): operator
    // reordering, sparse rewrites, training-invariant code motion and the training subgraph
    const bool train = std::getenv("GALA_REFGEN_TRAIN") != nullptr;
    const bool motion = train || std::getenv("GALA_REFGEN_CODE_MOTION") != nullptr;
    if (train) s.validation = 5;   // the corpus's validation_step=5 (tests/GALA-DSL/*)
    if (s.model == "gcn" || s.model == "gcn3") {  // gcn3: three layers (config 5's GCN-3, the
        s.layers = s.model == "gcn3" ? 3 : 2;        // tests/GALA-DSL/ablations/scalability shape)
        buildGcn(s);
    } else if (s.model == "gat") {
        if (!s.col_tile) {  // the generator's edge operators need the tiled graph (common.h:641-650)
            std::cerr << "gat: the reference generator supports the edge operators on a col_tile graph only\n";
            return 2;
        }
        buildGat(s);
    } else if (s.model == "gin") {
        buildGin(s);
    } else if (s.model == "sage") {
        buildSage(s);
    } else {
        std::cerr << "unknown model " << s.model << "\n";
        return 2;
    }
    auto *ctx = new GALAContext(GPU_DEVICE, SINGLE_NODE_SINGLE);
    auto gen = HIPGenerator(ctx, out);
    if (GALAFEContext::operator_reordering)
        GALATransformations::complexityOperatorReordering(GALAFEContext::program, GALAFEContext::dependencies,
                                                          GALAFEContext::associations, GALAFEContext::transforms);
    if (GALAFEContext::sparse_rewrites)
        GALATransformations::sparsityAwareRewrites(GALAFEContext::program, GALAFEContext::dependencies,
                                                   GALAFEContext::associations, GALAFEContext::transforms);
    if (motion)  // gala_train's third pass (tests/gala_train.cpp:136-140)
        GALATransformations::trainingInvariantCodeMotion(GALAFEContext::program, GALAFEContext::dependencies,
                                                         GALAFEContext::associations, GALAFEContext::transforms);
    if (train)  // gala_train's fourth pass (tests/gala_train.cpp:142-146)
        GALATransformations::trainingSubGraph(GALAFEContext::program, GALAFEContext::dependencies,
                                              GALAFEContext::associations, GALAFEContext::transforms);
    gen.writeCode(GALAFEContext::program, GALAFEContext::dependencies, GALAFEContext::associations,
                  GALAFEContext::transforms);
    std::cout << "wrote " << out << "gala.cu and " << out << "CMakeLists.txt" << std::endl;
    return 0;
}
