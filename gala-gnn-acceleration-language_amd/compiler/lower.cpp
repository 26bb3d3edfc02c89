// lower.cpp — DSL parse tree -> galac IR (ir.h).
//
// The reference's front-end classifies each layer statement into a LayerOpType by its
// syntactic shape (frontend.y:82-170, 238-290) and then instantiates fixed templates per
// op (addDegrees_CIR ... add_addTwoFFN_CIR, frontend.y:440-1000).  galac evaluates the
// layer body instead: every expression yields a symbolic value (graph, node features,
// node vector, edge values, function, number), and each operation appends one SSA node.
// The programs of tests/GALA-DSL lower to the same op sequences the reference builds:
//   GCN  DEGREES, POWER(-0.5), ROW_BROADCAST, AGGREGATE, FFN, ROW_BROADCAST, RELU
//   GAT  FFN, FFN(out=1) x2, AGGREGATE_EDGE_SUM + LEAKY_RELU(0.2), SOFTMAX, AGGREGATE
//   GIN  AGGREGATE, SCALAR_ADD_EPS_MULTIPLY, ADD, FFN, RELU
//   SAGE DEGREES, POWER(-1), AGGREGATE, ROW_BROADCAST (= mul_mean), FFN, FFN(self), ADD
// Two reference behaviours are kept on purpose:
//   - `dsl.fn.softmax(G, attn)` over the output of an edge aggregation gets the
//     LeakyReLU(0.2) the reference inserts (frontend.y:1000-1003, addLeakyReLU);
//   - a name read in a layer before it is assigned (SAGE's `dsl.nn.ffn(res, out=hs)`)
//     denotes the layer's input features, which is what ADD_TWO_FFN's self FFN reads
//     (frontend.y:163-167, add_addTwoFFN_CIR).
#include <algorithm>
#include <cstring>
#include <fstream>
#include <functional>
#include <map>
#include <sstream>
#include <vector>

#include "../host/gala_datasets.h"
#include "ir.h"

namespace galac {

namespace {
// .npy header: dtype descr and shape; `data` at the first element (little-endian, C order)
struct NpyHead {
    std::string descr;
    std::vector<int64_t> shape;
    std::streamoff data = 0;
};

bool npy_head(const std::string &path, NpyHead *out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    char magic[8];
    if (!f.read(magic, 8) || std::memcmp(magic, "\x93NUMPY", 6) != 0) return false;
    uint32_t hlen = 0;
    if (magic[6] == 1) {
        uint16_t h16 = 0;
        f.read((char *)&h16, 2);
        hlen = h16;
    } else {
        f.read((char *)&hlen, 4);
    }
    std::string h(hlen, ' ');
    if (!f.read(&h[0], hlen)) return false;
    auto field = [&](const char *key) {
        const size_t k = h.find(std::string("'") + key + "'");
        if (k == std::string::npos) return std::string();
        size_t a = h.find(':', k) + 1;
        while (a < h.size() && h[a] == ' ') ++a;
        const char close = h[a] == '(' ? ')' : (h[a] == '\'' ? '\'' : ',');
        const size_t b = h.find(close, a + 1);
        return h.substr(a, b == std::string::npos ? std::string::npos : b - a + 1);
    };
    out->descr = field("descr");
    if (out->descr.size() < 4 || out->descr[1] == '>' || field("fortran_order").find("True") != std::string::npos)
        return false;
    out->descr = out->descr.substr(2, out->descr.size() - 3);   // '<u4' -> u4
    const std::string shp = field("shape");
    for (size_t q = 0; q < shp.size();) {
        if (!std::isdigit((unsigned char)shp[q])) { ++q; continue; }
        size_t e = q;
        while (e < shp.size() && std::isdigit((unsigned char)shp[e])) ++e;
        out->shape.push_back(std::stoll(shp.substr(q, e - q)));
        q = e;
    }
    out->data = (std::streamoff)(magic[6] == 1 ? 10 : 12) + hlen;
    return true;
}

// The dataset facts gala_inference reads at compile time (tests/gala_inference.cpp:98-120):
// readSM_npy32's rows (Adj_src[0]) and stored edges (Adj_dst's length, tests/common.h:
// 331-366), Feat.npy's columns and max(Lab) + 1.  false when a file is missing or unreadable.
bool read_dataset_facts(const std::string &dir, int64_t *nrows, int64_t *nvals, int64_t *feat, int64_t *classes) {
    NpyHead src, dst, ft, lab;
    if (!npy_head(dir + "Adj_src.npy", &src) || !npy_head(dir + "Adj_dst.npy", &dst) ||
        !npy_head(dir + "Feat.npy", &ft) || !npy_head(dir + "Lab.npy", &lab))
        return false;
    if (src.descr != "u4" || src.shape.empty() || src.shape[0] < 2 || dst.shape.empty() || ft.shape.size() != 2)
        return false;
    std::ifstream fs(dir + "Adj_src.npy", std::ios::binary);
    uint32_t head[2];
    fs.seekg(src.data);
    if (!fs.read((char *)head, sizeof(head))) return false;
    *nrows = head[0];
    *nvals = dst.shape[0];
    *feat = ft.shape[1];
    int64_t n = 1;
    for (int64_t d : lab.shape) n *= d;
    std::ifstream fl(dir + "Lab.npy", std::ios::binary);
    fl.seekg(lab.data);
    int64_t mx = -1;
    if (lab.descr == "i8") {
        std::vector<int64_t> v((size_t)n);
        if (!fl.read((char *)v.data(), (std::streamsize)(n * 8))) return false;
        for (int64_t x : v) mx = std::max(mx, x);
    } else if (lab.descr == "i4") {
        std::vector<int32_t> v((size_t)n);
        if (!fl.read((char *)v.data(), (std::streamsize)(n * 4))) return false;
        for (int32_t x : v) mx = std::max<int64_t>(mx, x);
    } else {
        return false;
    }
    *classes = mx + 1;
    return true;
}
}  // namespace

const char *op_name(Op op) {
    switch (op) {
    case Op::Input: return "INPUT";
    case Op::Degrees: return "DEGREES";
    case Op::SampledDegrees: return "FULL";
    case Op::Power: return "POWER";
    case Op::RowBroadcast: return "ROW_BROADCAST";
    case Op::Aggregate: return "AGGREGATE_MUL_SUM";
    case Op::Ffn: return "FFN";
    case Op::Relu: return "RELU";
    case Op::EdgeAdd: return "AGGREGATE_EDGE_SUM";
    case Op::LeakyRelu: return "LEAKY_RELU";
    case Op::Softmax: return "SOFTMAX";
    case Op::ScaleEps: return "SCALAR_ADD_EPS_MULTIPLY";
    case Op::Add: return "ADD";
    case Op::EdgeMul: return "AGGREGATE_EDGE_MUL";
    case Op::GcnAggregate: return "GCN_AGGREGATE";
    case Op::GatAggregate: return "GAT_AGGREGATE";
    }
    return "?";
}

int Module::add_value(const std::string &name, Kind k, int64_t width, bool invariant) {
    values.push_back({name, k, width, invariant});
    return (int)values.size() - 1;
}

int Module::add_node(Node n) {
    nodes.push_back(n);
    return (int)nodes.size() - 1;
}

std::vector<int> Module::uses(int value) const {
    std::vector<int> u;
    for (int i = 0; i < (int)nodes.size(); ++i) {
        if (nodes[i].dead) continue;
        for (int v : nodes[i].in)
            if (v == value) {
                u.push_back(i);
                break;
            }
    }
    return u;
}

int Module::producer(int value) const {
    for (int i = 0; i < (int)nodes.size(); ++i)
        if (!nodes[i].dead && nodes[i].out == value) return i;
    return -1;
}

std::string Module::dump() const {
    std::ostringstream o;
    auto vname = [&](int v) {
        return v < 0 ? std::string("-") : "%" + std::to_string(v) + ":" + values[v].name;
    };
    for (int pass = 0; pass < 2; ++pass) {
        o << (pass == 0 ? "invariant:\n" : "training loop:\n");
        for (const Node &n : nodes) {
            if (n.dead || n.hoisted != (pass == 0)) continue;
            o << "  " << vname(n.out) << "[" << values[n.out].width << "] = " << op_name(n.op)
              << "(";
            for (size_t i = 0; i < n.in.size(); ++i) o << (i ? ", " : "") << vname(n.in[i]);
            o << ")";
            if (n.op == Op::Power || n.op == Op::LeakyRelu || n.op == Op::ScaleEps)
                o << " param=" << n.param;
            if (n.weight >= 0)
                o << " w=" << weights[n.weight].name << "[" << weights[n.weight].in << "x"
                  << weights[n.weight].out << (weights[n.weight].heads > 1 ? " per head" : "") << "]";
            if (n.op == Op::Aggregate || n.op == Op::GcnAggregate || n.op == Op::GatAggregate)
                o << " graph=" << n.graph;
            if (n.layer >= 0) o << " layer=" << n.layer;
            o << "\n";
        }
    }
    o << "output: " << vname(output) << "\n";
    return o.str();
}

std::string Module::to_json() const {
    std::ostringstream o;
    auto str = [](const std::string &x) {
        std::string r = "\"";
        for (char ch : x) {
            if (ch == '"' || ch == '\\') r += '\\';
            r += ch;
        }
        return r + "\"";
    };
    o.precision(17);
    const Schedule &s = sched;
    o << "{\"source\": " << str(source) << ", \"output\": " << output
      << ", \"num_graphs\": " << num_graphs << ", \"num_layers\": " << num_layers
      << ",\n \"sched\": {\"dataset\": " << str(s.dataset) << ", \"opt_input\": " << str(s.opt_input)
      << ", \"unweighted\": " << s.unweighted << ", \"coarsen\": " << s.coarsen << ", \"undirected\": " << s.undirected
      << ", \"sparse\": " << s.sparse << ", \"feat_size\": " << s.feat_size
      << ", \"label_size\": " << s.label_size << ", \"col_tile\": " << s.col_tile
      << ", \"data_sample\": " << s.data_sample << ", \"kernel_sample\": " << s.kernel_sample
      << ", \"dynamic_sample\": " << s.dynamic_sample << ", \"iterations\": " << s.iterations
      << ", \"gat_mode\": " << s.gat_mode << ", \"gat_heads\": " << s.gat_heads << "},\n \"weights\": [";
    for (size_t k = 0; k < weights.size(); ++k)
        o << (k ? ", " : "") << "{\"name\": " << str(weights[k].name) << ", \"type\": "
          << (weights[k].type == Weight::Linear ? "\"linear\"" : "\"eps\"") << ", \"in\": "
          << weights[k].in << ", \"out\": " << weights[k].out << ", \"init\": " << weights[k].init
          << ", \"heads\": " << weights[k].heads << "}";
    o << "],\n \"values\": [";
    for (size_t k = 0; k < values.size(); ++k) {
        const Value &v = values[k];
        o << (k ? ", " : "") << "{\"name\": " << str(v.name) << ", \"kind\": \""
          << (v.kind == Kind::Node ? "node" : v.kind == Kind::NodeVec ? "nodevec"
                                             : v.kind == Kind::Edge ? "edge" : "scalar")
          << "\", \"width\": " << v.width << "}";
    }
    o << "],\n \"nodes\": [";
    bool first = true;
    for (const Node &n : nodes) {
        if (n.dead) continue;
        o << (first ? "\n  " : ",\n  ") << "{\"op\": \"" << op_name(n.op) << "\", \"in\": [";
        first = false;
        for (size_t k = 0; k < n.in.size(); ++k) o << (k ? ", " : "") << n.in[k];
        o << "], \"out\": " << n.out << ", \"param\": " << n.param << ", \"weight\": "
          << (n.weight >= 0 ? str(weights[n.weight].name) : std::string("null"))
          << ", \"graph\": " << n.graph << ", \"layer\": " << n.layer
          << ", \"hoisted\": " << (n.hoisted ? "true" : "false") << "}";
    }
    o << "]}\n";
    return o.str();
}

namespace {

struct LayerDef {
    std::string name;
    std::vector<std::string> params;
    std::vector<StmtP> body;
    SrcLoc at;
};

// A symbolic value during evaluation.
struct Sym {
    enum T { None, Graph, Graphs, Val, AggrFn, EdgeFn, NonLn, Num, Scalar, Str, Bool, Null };
    T t = None;
    int val = -1;               // Val: IR value id
    double num = 0;
    bool is_int = false;
    std::string s;              // Str; AggrFn semiring ("mul_sum"/"mul_mean")
    int nonln = 0;              // NonLn: 0 identity (null), 1 ReLU, 2 LeakyReLU
    static Sym of_val(int v) {
        Sym x;
        x.t = Val;
        x.val = v;
        return x;
    }
};

class Lowering {
  public:
    explicit Lowering(const Program &p) : prog_(p) { m_.source = p.source_name; }

    Module run() {
        for (const StmtP &st : prog_.stmts) top(*st);
        if (m_.sched.dataset.empty())
            throw DslError({1, 1}, "program does not load a dataset (G = load_dataset(\"...\"))");
        if (model_inst_.empty()) throw DslError({1, 1}, "program does not instantiate a model");
        build_model();
        return std::move(m_);
    }

  private:
    const Program &prog_;
    Module m_;
    std::string graph_var_;
    std::map<std::string, std::string> aggr_fns_;   // var -> semiring
    std::map<std::string, bool> edge_fns_;
    std::map<std::string, LayerDef> layers_;
    std::map<std::string, LayerDef> models_;
    std::string model_inst_, model_def_;
    ExprP model_call_;
    int input_ = -1;
    std::map<std::string, int> graph_cache_;  // hoistable graph values shared by layers

    // ---- top level -------------------------------------------------------------------
    static std::string callee_path(const Expr &e) {
        return e.kind == Expr::Call && e.obj ? e.obj->path() : std::string();
    }
    static const Expr *arg(const Expr &call, size_t i, const char *kw = nullptr) {
        if (kw)
            for (size_t k = 0; k < call.args.size(); ++k)
                if (call.kw[k] == kw) return call.args[k].get();
        size_t pos = 0;
        for (size_t k = 0; k < call.args.size(); ++k) {
            if (!call.kw[k].empty()) continue;
            if (pos++ == i) return call.args[k].get();
        }
        return nullptr;
    }
    static int64_t int_arg(const Expr &call, size_t i, const char *what) {
        const Expr *a = arg(call, i);
        if (!a || a->kind != Expr::Number || !a->is_int)
            throw DslError(call.at, std::string(what) + " expects an integer");
        return (int64_t)a->num;
    }
    static bool bool_arg(const Expr &call, const char *what) {
        const Expr *a = arg(call, 0);
        if (!a || a->kind != Expr::Bool) throw DslError(call.at, std::string(what) + " expects true/false");
        return a->bval;
    }

    void top(const Stmt &st) {
        if (st.kind == Stmt::Block) {
            LayerDef d{st.block_name, st.params, st.body, st.at};
            if (st.block_kind == "layer") layers_[st.block_name] = d;
            else models_[st.block_name] = d;
            return;
        }
        const Expr &v = *st.value;
        if (st.kind == Stmt::Eval) {
            top_call(v);
            return;
        }
        const std::string target = st.target->path();
        const std::string cp = callee_path(v);
        if (cp == "load_dataset") {
            const Expr *a = arg(v, 0);
            if (!a || a->kind != Expr::String) throw DslError(v.at, "load_dataset expects a name");
            m_.sched.dataset = a->name;
            graph_var_ = target;
            return;
        }
        if (cp == "dsl.get_aggregate" || cp == "dsl.get_edge_aggregate") {
            const Expr *f = arg(v, 0, "fn");
            const std::string fp = f ? f->path() : "";
            if (cp == "dsl.get_aggregate") {
                if (fp != "dsl.fn.mul_sum" && fp != "dsl.fn.mul_mean")
                    throw DslError(v.at, "get_aggregate supports fn = dsl.fn.mul_sum | dsl.fn.mul_mean");
                aggr_fns_[target] = fp.substr(7);
            } else {
                if (fp != "dsl.fn.sum") throw DslError(v.at, "get_edge_aggregate supports fn = dsl.fn.sum");
                edge_fns_[target] = true;
            }
            return;
        }
        if (v.kind == Expr::Call && v.obj && v.obj->kind == Expr::Ident &&
            models_.count(v.obj->name)) {
            model_inst_ = target;
            model_def_ = v.obj->name;
            model_call_ = st.value;
            return;
        }
        // m1.eval()
        if (v.kind == Expr::Call && v.obj && v.obj->kind == Expr::Member &&
            v.obj->name == "eval" && v.obj->obj && v.obj->obj->path() == model_inst_)
            return;
        // schedule: G = G.method(...)
        if (target == graph_var_ && !graph_var_.empty() && v.kind == Expr::Call && v.obj &&
            v.obj->kind == Expr::Member && v.obj->obj && v.obj->obj->path() == graph_var_) {
            graph_schedule(v, v.obj->name);
            return;
        }
        // schedule: aggrFn = aggrFn.coarsen(n) | .sample(n) | .sample(n).dynamic()
        if (aggr_fns_.count(target) && v.kind == Expr::Call) {
            fn_schedule(v, target);
            return;
        }
        throw DslError(st.at, "unsupported statement assigning '" + target + "'");
    }

    void graph_schedule(const Expr &call, const std::string &method) {
        Schedule &s = m_.sched;
        if (method == "set_undirected") s.undirected = bool_arg(call, "set_undirected");
        else if (method == "set_unweighted") s.unweighted = bool_arg(call, "set_unweighted");
        else if (method == "is_sparser") s.sparse = bool_arg(call, "is_sparser");
        else if (method == "col_tile") s.col_tile = int_arg(call, 0, "col_tile");
        else if (method == "sample") s.data_sample = int_arg(call, 0, "sample");
        else if (method == "opt_input") {
            const Expr *a = arg(call, 0);
            if (!a || a->kind != Expr::String) throw DslError(call.at, "opt_input expects a path");
            s.opt_input = a->name;
        } else {
            throw DslError(call.at, "unknown graph transformation '" + method + "'");
        }
    }

    void fn_schedule(const Expr &v, const std::string &fn) {
        const Expr *c = &v;
        bool dynamic = false;
        if (c->obj && c->obj->kind == Expr::Member && c->obj->name == "dynamic") {
            dynamic = true;
            c = c->obj->obj.get();
            if (!c || c->kind != Expr::Call) throw DslError(v.at, "expected .sample(n).dynamic()");
        }
        if (!c->obj || c->obj->kind != Expr::Member || c->obj->obj->path() != fn)
            throw DslError(v.at, "expected " + fn + "." + "<transformation>(...)");
        const std::string method = c->obj->name;
        if (method == "coarsen" && !dynamic) {
            m_.sched.coarsen = int_arg(*c, 0, "coarsen");
        } else if (method == "sample") {
            m_.sched.kernel_sample = int_arg(*c, 0, "sample");
            m_.sched.dynamic_sample = dynamic;
        } else {
            throw DslError(v.at, "unknown compute transformation '" + method + "'");
        }
    }

    void top_call(const Expr &v) {
        const std::string cp = callee_path(v);
        Schedule &s = m_.sched;
        if (cp == model_inst_ + ".train" && !model_inst_.empty()) {
            for (size_t k = 0; k < v.args.size(); ++k) {
                const Expr &a = *v.args[k];
                if (a.kind != Expr::Number || !a.is_int)
                    throw DslError(a.at, "train() arguments are integers");
                if (v.kw[k] == "iters") s.iterations = (int64_t)a.num;
                else if (v.kw[k] == "validation_step") s.validation_step = (int64_t)a.num;
                else throw DslError(a.at, "unknown train() argument '" + v.kw[k] + "'");
            }
            return;
        }
        if (cp == "feature_size") s.feat_size = int_arg(v, 0, "feature_size");
        else if (cp == "label_size") s.label_size = int_arg(v, 0, "label_size");
        else if (cp == "print_accuracy") s.print_accuracy = bool_arg(v, "print_accuracy");
        else if (cp == "print_memory") s.print_memory = bool_arg(v, "print_memory");
        else if (cp == "operator_reordering") s.operator_reordering = bool_arg(v, "operator_reordering");
        else if (cp == "sparse_rewrites") s.sparse_rewrites = bool_arg(v, "sparse_rewrites");
        else if (cp == "training_subgraph") s.training_subgraph = bool_arg(v, "training_subgraph");
        else if (cp == "train_code_motion") s.train_code_motion = bool_arg(v, "train_code_motion");
        // galac extension: exact GAT gradients (GALA_SOFTMAX_FIXED) instead of the
        // reference's backward chain
        else if (cp == "gat_fixed_gradients") s.gat_mode = bool_arg(v, "gat_fixed_gradients") ? 1 : 0;
        // galac extension: multi-head attention (the reference DSL is single-head,
        // frontend.y:987-1008); BASELINE's 8-head GAT is gat_heads(8)
        else if (cp == "gat_heads") {
            s.gat_heads = int_arg(v, 0, "gat_heads");
            if (s.gat_heads < 1 || s.gat_heads > 64) throw DslError(v.at, "gat_heads(H) needs 1 <= H <= 64");
        }
        else throw DslError(v.at, "unsupported statement '" + (cp.empty() ? std::string("?") : cp) + "'");
    }

    // ---- model -----------------------------------------------------------------------
    int64_t labels() const {
        if (m_.sched.label_size <= 0)
            throw DslError({1, 1}, "G.labels.size() needs label_size(n) in the schedule");
        return m_.sched.label_size;
    }

    // G.opt_input(path): the input-aware schedule gala_inference fixes after parsing
    // (tests/gala_inference.cpp:84-131) -- undirected, unweighted, coarsen(2), the feature and
    // label sizes of the dataset, and COL_TILE nrows / 5 when nnz / nrows^2 > 0.001.  The
    // facts come from the dataset's files (the path as written, from the working directory as
    // the reference opens it, else from the DSL file's directory); when neither holds them,
    // from the dataset's published shape (nnz = 2 * undirected edges + N self loops, the
    // export's normalisation), noted.  The reference would stop there instead.
    void auto_schedule() {
        Schedule &s = m_.sched;
        int64_t nrows = 0, nvals = 0, feat = 0, classes = 0;
        // the reference joins the file names straight onto the path as written
        // (gala_inference.cpp:102-117, common.h:342), so a prefix ("data/reddit_") is tried
        // first as it stands, then as a directory ('/' added), then from the DSL file's directory
        const std::string asis = s.opt_input;
        std::string dir = asis;
        if (!dir.empty() && dir.back() != '/') dir += '/';
        std::string from;
        const std::string src_dir = m_.source.find('/') == std::string::npos
                                        ? std::string()
                                        : m_.source.substr(0, m_.source.rfind('/') + 1);
        const bool rel = !asis.empty() && asis[0] != '/';
        if (!asis.empty() && read_dataset_facts(asis, &nrows, &nvals, &feat, &classes)) {
            from = "the files at " + asis;
        } else if (read_dataset_facts(dir, &nrows, &nvals, &feat, &classes)) {
            from = "the files in " + dir;
        } else if (!src_dir.empty() && rel && read_dataset_facts(src_dir + asis, &nrows, &nvals, &feat, &classes)) {
            from = "the files at " + src_dir + asis;
        } else if (!src_dir.empty() && rel &&
                   read_dataset_facts(src_dir + dir, &nrows, &nvals, &feat, &classes)) {
            from = "the files in " + src_dir + dir;
        } else {
            gala::DatasetShape shape{};
            if (!gala::dataset_shape(s.dataset, &shape))
                throw DslError({1, 1}, "opt_input(\"" + s.opt_input + "\"): no dataset files there and no published "
                                       "shape for '" + s.dataset + "'");
            nrows = shape.n;
            nvals = 2 * shape.undirected + shape.n;
            feat = shape.feat;
            classes = shape.classes;
            from = "the published " + s.dataset + " shape (no dataset files at " + s.opt_input + ")";
        }
        s.undirected = true;
        s.unweighted = true;
        s.coarsen = 2;
        s.feat_size = feat;
        s.label_size = classes;
        // ((float)nvals / ((long)nrows * nrows)) > 0.001, as the reference evaluates it
        const float density = (float)nvals / (float)(nrows * nrows);
        if ((double)density > 0.001) s.col_tile = nrows / 5;
        std::ostringstream o;
        o << "opt_input schedule from " << from << ": N=" << nrows << " nnz=" << nvals << " density=" << density
          << " -> undirected, unweighted, coarsen(2), feature_size " << feat << ", label_size " << classes
          << (s.col_tile ? ", col_tile(" + std::to_string(s.col_tile) + ")" : std::string(", no column tiling"));
        m_.notes.push_back(o.str());
    }

    void build_model() {
        if (!m_.sched.opt_input.empty()) auto_schedule();
        // sizes not given in the schedule: the dataset's published shape (the reference's
        // gala_inference reads them from the files at compile time, gala_inference.cpp:84-130)
        gala::DatasetShape shape{};
        const bool known = gala::dataset_shape(m_.sched.dataset, &shape);
        if (m_.sched.feat_size <= 0 && known) {
            m_.sched.feat_size = shape.feat;
            m_.notes.push_back("feature_size from the " + m_.sched.dataset + " shape: " + std::to_string(shape.feat));
        }
        if (m_.sched.label_size <= 0 && known) {
            m_.sched.label_size = shape.classes;
            m_.notes.push_back("label_size from the " + m_.sched.dataset + " shape: " + std::to_string(shape.classes));
        }
        if (m_.sched.feat_size <= 0)
            throw DslError({1, 1}, "the schedule must give feature_size(n) for dataset '" +
                                       m_.sched.dataset + "'");
        const LayerDef &md = models_.at(model_def_);
        // bind model params to the instance's arguments
        std::map<std::string, Sym> menv;
        const Expr &mc = *model_call_;
        for (size_t i = 0; i < md.params.size(); ++i) {
            const Expr *a = arg(mc, i);
            if (!a) throw DslError(mc.at, "model " + md.name + " expects " +
                                              std::to_string(md.params.size()) + " arguments");
            menv[md.params[i]] = top_sym(*a);
        }
        input_ = m_.add_value("t_iden", Kind::Node, m_.sched.feat_size, true);
        Node in{Op::Input};
        in.out = input_;
        in.hoisted = true;
        m_.add_node(in);
        std::map<std::string, int> layer_out;
        int layer = 0;
        // count layers first (the last one's nonln / label width)
        for (const StmtP &st : md.body)
            if (st->kind != Stmt::Assign || st->value->kind != Expr::Call)
                throw DslError(st->at, "a model body holds `lk = Layer(...)` statements");
        m_.num_layers = (int)md.body.size();
        for (const StmtP &st : md.body) {
            const Expr &call = *st->value;
            const std::string lname = call.obj ? call.obj->path() : "";
            auto it = layers_.find(lname);
            if (it == layers_.end()) throw DslError(call.at, "unknown layer '" + lname + "'");
            const LayerDef &ld = it->second;
            if (call.args.size() != ld.params.size())
                throw DslError(call.at, "layer " + lname + " expects " +
                                            std::to_string(ld.params.size()) + " arguments");
            std::map<std::string, Sym> env;
            int feats = -1;
            for (size_t i = 0; i < ld.params.size(); ++i) {
                const Expr &a = *call.args[i];
                Sym s;
                const std::string ap = a.path();
                if (a.kind == Expr::Ident && layer_out.count(a.name)) {
                    s.t = Sym::Graph;  // a previous layer: the graph with its features
                    feats = layer_out[a.name];
                } else if (a.kind == Expr::Ident && menv.count(a.name)) {
                    s = menv[a.name];
                    if (s.t == Sym::Graph) feats = input_;
                } else if (a.kind == Expr::Call && callee_path(a) == graph_var_ + ".labels.size") {
                    s.t = Sym::Num;
                    s.num = (double)labels();
                    s.is_int = true;
                } else if (a.kind == Expr::Call && a.obj && a.obj->kind == Expr::Member &&
                           a.obj->name == "size" && a.obj->obj &&
                           a.obj->obj->kind == Expr::Member && a.obj->obj->name == "labels") {
                    s.t = Sym::Num;
                    s.num = (double)labels();
                    s.is_int = true;
                } else {
                    s = top_sym(a);
                    if (s.t == Sym::Graph) feats = input_;
                    (void)ap;
                }
                env[ld.params[i]] = s;
            }
            if (feats < 0) throw DslError(call.at, "layer call passes no graph / previous layer");
            layer_out[st->target->path()] = lower_layer(ld, env, feats, layer);
            ++layer;
        }
        m_.output = layer_out[md.body.back()->target->path()];
    }

    Sym top_sym(const Expr &a) {
        Sym s;
        const std::string p = a.path();
        if (a.kind == Expr::Null) {
            s.t = Sym::NonLn;
            s.nonln = 0;
        } else if (p == "dsl.non_ln.ReLU") {
            s.t = Sym::NonLn;
            s.nonln = 1;
        } else if (p == "dsl.non_ln.LeakyReLU") {
            s.t = Sym::NonLn;
            s.nonln = 2;
        } else if (!p.empty() && p == graph_var_) {
            s.t = Sym::Graph;
        } else if (aggr_fns_.count(p)) {
            s.t = Sym::AggrFn;
            s.s = aggr_fns_[p];
        } else if (edge_fns_.count(p)) {
            s.t = Sym::EdgeFn;
        } else if (a.kind == Expr::Number) {
            s.t = Sym::Num;
            s.num = a.num;
            s.is_int = a.is_int;
        } else if (a.kind == Expr::Bool) {
            s.t = Sym::Bool;
            s.num = a.bval;
        } else {
            throw DslError(a.at, "cannot pass '" + (p.empty() ? std::string("expression") : p) +
                                     "' to a model or layer");
        }
        return s;
    }

    // ---- layer body ------------------------------------------------------------------
    struct LayerCtx {
        const LayerDef *def;
        std::map<std::string, Sym> env;  // params + locals
        std::string gname;               // the layer's graph parameter
        int feats = -1;                  // G.node.feats
        int in_feats = -1;
        int edge_vals = -1;              // G.edges.vals once assigned
        int layer = 0;
        bool last = false;
        int64_t heads = 1;               // attention heads of this layer (gat_heads)
    };

    int node(Op op, std::vector<int> in, const std::string &name, Kind k, int64_t width,
             LayerCtx &c, double param = 0, int weight = -1) {
        bool inv = weight < 0 && op != Op::ScaleEps;
        for (int v : in)
            if (v >= 0) inv = inv && m_.values[v].invariant;
        const int out = m_.add_value(name, k, width, inv);
        Node n{op};
        n.in = std::move(in);
        n.out = out;
        n.param = param;
        n.weight = weight;
        n.layer = c.layer;
        m_.add_node(n);
        return out;
    }

    int graph_value(Op op, double param, int input, LayerCtx &c) {
        // DEGREES / POWER of the graph: the same values for every layer (the reference
        // emits them in layer 0 only, frontend.y:950-960)
        const std::string key = std::string(op_name(op)) + "/" + std::to_string(param) + "/" +
                                std::to_string(input);
        auto it = graph_cache_.find(key);
        if (it != graph_cache_.end()) return it->second;
        int v;
        if (op == Op::Degrees) {
            if (m_.sched.kernel_sample > 0)
                v = node(Op::SampledDegrees, {}, "degrees", Kind::NodeVec, 1, c,
                         (double)m_.sched.kernel_sample);
            else
                v = node(Op::Degrees, {}, "degrees", Kind::NodeVec, 1, c);
        } else {
            v = node(Op::Power, {input}, "norm", Kind::NodeVec, 1, c, param);
        }
        m_.nodes.back().layer = -1;
        graph_cache_[key] = v;
        return v;
    }

    int new_weight(const std::string &prefix, int64_t in, int64_t out) {
        int k = 0;
        for (const Weight &w : m_.weights)
            if (w.name.rfind(prefix, 0) == 0) ++k;
        m_.weights.push_back({prefix + std::to_string(k), Weight::Linear, in, out, 0});
        return (int)m_.weights.size() - 1;
    }

    int as_val(const Sym &s, const Expr &at, const char *what) {
        if (s.t != Sym::Val) throw DslError(at.at, std::string(what) + " expects a tensor");
        return s.val;
    }

    int lower_layer(const LayerDef &ld, std::map<std::string, Sym> env, int feats, int layer) {
        LayerCtx c;
        c.def = &ld;
        c.env = std::move(env);
        c.feats = c.in_feats = feats;
        c.layer = layer;
        c.last = layer == m_.num_layers - 1;
        bool attention = false;
        for (const auto &kv : c.env) {
            if (kv.second.t == Sym::Graph) c.gname = kv.first;
            attention = attention || kv.second.t == Sym::EdgeFn;
        }
        // multi-head attention in every attention layer but the output layer (one head:
        // the standard GAT output, BASELINE config 3's layer 2)
        c.heads = (attention && !c.last) ? m_.sched.gat_heads : 1;
        if (c.gname.empty()) throw DslError(ld.at, "layer " + ld.name + " has no graph parameter");
        int out = -1;
        for (const StmtP &st : ld.body) {
            if (st->kind == Stmt::Block) throw DslError(st->at, "nested definitions are not allowed");
            Sym v = eval(*st->value, c);
            if (st->kind == Stmt::Eval) continue;
            const std::string t = st->target->path();
            if (t == c.gname + ".node.feats") {
                c.feats = as_val(v, *st->value, "G.node.feats =");
                out = c.feats;
            } else if (t == c.gname + ".edges.vals") {
                const int e = as_val(v, *st->value, "G.edges.vals =");
                if (m_.values[e].kind != Kind::Edge)
                    throw DslError(st->at, "G.edges.vals needs edge values");
                c.edge_vals = e;
            } else if (st->target->kind == Expr::Ident) {
                c.env[t] = v;
                if (v.t == Sym::Val) m_.values[v.val].name = t;
            } else {
                throw DslError(st->at, "cannot assign to '" + t + "'");
            }
        }
        if (out < 0) throw DslError(ld.at, "layer " + ld.name + " never sets G.node.feats");
        return out;
    }

    Sym eval(const Expr &e, LayerCtx &c) {
        switch (e.kind) {
        case Expr::Number: {
            Sym s;
            s.t = Sym::Num;
            s.num = e.num;
            s.is_int = e.is_int;
            return s;
        }
        case Expr::String: {
            Sym s;
            s.t = Sym::Str;
            s.s = e.name;
            return s;
        }
        case Expr::Null: {
            Sym s;
            s.t = Sym::NonLn;
            return s;
        }
        case Expr::Bool: {
            Sym s;
            s.t = Sym::Bool;
            s.num = e.bval;
            return s;
        }
        case Expr::Ident: {
            auto it = c.env.find(e.name);
            if (it != c.env.end()) return it->second;
            // read before assignment: the layer's input features (see header)
            m_.notes.push_back("layer " + std::to_string(c.layer) + ": '" + e.name +
                               "' read before assignment -> the layer's input features");
            return Sym::of_val(c.in_feats);
        }
        case Expr::Member: {
            const std::string p = e.path();
            if (p == c.gname + ".node.feats") return Sym::of_val(c.feats);
            if (p == c.gname + ".graphs" || p == c.gname) {
                Sym s;
                s.t = p == c.gname ? Sym::Graph : Sym::Graphs;
                return s;
            }
            if (p == c.gname + ".edges.vals") {
                if (c.edge_vals < 0) throw DslError(e.at, "G.edges.vals read before it is set");
                return Sym::of_val(c.edge_vals);
            }
            if (p == "dsl.non_ln.ReLU" || p == "dsl.non_ln.LeakyReLU") {
                Sym s;
                s.t = Sym::NonLn;
                s.nonln = p == "dsl.non_ln.ReLU" ? 1 : 2;
                return s;
            }
            throw DslError(e.at, "unknown name '" + p + "'");
        }
        case Expr::Neg: {
            Sym v = eval(*e.obj, c);
            if (v.t != Sym::Num) throw DslError(e.at, "unary minus needs a number");
            v.num = -v.num;
            return v;
        }
        case Expr::Binary: return binary(e, c);
        case Expr::Call: return call(e, c);
        }
        throw DslError(e.at, "unsupported expression");
    }

    Sym binary(const Expr &e, LayerCtx &c) {
        Sym a = eval(*e.lhs, c), b = eval(*e.rhs, c);
        if (e.name == "*") {
            if (a.t == Sym::Scalar || b.t == Sym::Scalar) {
                const Sym &s = a.t == Sym::Scalar ? a : b;
                const Sym &x = a.t == Sym::Scalar ? b : a;
                const int xv = as_val(x, e, "scalar *");
                const int w = (int)m_.weights.size();
                int k = 0;
                for (const Weight &ww : m_.weights) k += ww.type == Weight::Eps;
                m_.weights.push_back({"eps" + std::to_string(k), Weight::Eps, 1, 1, s.num});
                return Sym::of_val(node(Op::ScaleEps, {xv}, "res", Kind::Node,
                                        m_.values[xv].width, c, s.num, w));
            }
            const int av = as_val(a, e, "*"), bv = as_val(b, e, "*");
            const Kind ka = m_.values[av].kind, kb = m_.values[bv].kind;
            if (ka == Kind::NodeVec && kb == Kind::Node)
                return Sym::of_val(node(Op::RowBroadcast, {av, bv}, "res", Kind::Node,
                                        m_.values[bv].width, c));
            if (ka == Kind::Node && kb == Kind::NodeVec)
                return Sym::of_val(node(Op::RowBroadcast, {bv, av}, "res", Kind::Node,
                                        m_.values[av].width, c));
            throw DslError(e.at, "'*' multiplies a per-node vector (e.g. a norm) with features");
        }
        if (e.name == "+") {
            const int av = as_val(a, e, "+"), bv = as_val(b, e, "+");
            if (m_.values[av].kind != m_.values[bv].kind || m_.values[av].width != m_.values[bv].width)
                throw DslError(e.at, "'+' needs operands of the same shape (" +
                                         std::to_string(m_.values[av].width) + " vs " +
                                         std::to_string(m_.values[bv].width) + " columns)");
            return Sym::of_val(node(Op::Add, {av, bv}, "res", m_.values[av].kind,
                                    m_.values[av].width, c));
        }
        throw DslError(e.at, "operator '" + e.name + "' is not supported on tensors");
    }

    Sym call(const Expr &e, LayerCtx &c) {
        const std::string cp = e.obj ? e.obj->path() : "";
        // graph methods
        if (cp == c.gname + ".graphs.degrees" || cp == c.gname + ".degrees")
            return Sym::of_val(graph_value(Op::Degrees, 0, -1, c));
        if (cp == "dsl.fn.pow") {
            const Expr *x = arg(e, 0), *p = arg(e, 1);
            if (!x || !p) throw DslError(e.at, "pow(x, exponent)");
            Sym xs = eval(*x, c), ps = eval(*p, c);
            if (ps.t != Sym::Num) throw DslError(p->at, "pow exponent must be a number");
            const int xv = as_val(xs, *x, "pow");
            if (m_.values[xv].invariant && m_.values[xv].kind == Kind::NodeVec)
                return Sym::of_val(graph_value(Op::Power, ps.num, xv, c));
            return Sym::of_val(node(Op::Power, {xv}, "res", m_.values[xv].kind,
                                    m_.values[xv].width, c, ps.num));
        }
        if (cp == "dsl.nn.ffn") {
            const Expr *x = arg(e, 0), *o = arg(e, 1, "out");
            if (!x || !o) throw DslError(e.at, "ffn(x, out=n)");
            const int xv = as_val(eval(*x, c), *x, "ffn");
            Sym os = eval(*o, c);
            if (os.t != Sym::Num || !os.is_int || os.num < 1)
                throw DslError(o->at, "ffn out= must be a positive integer");
            const int64_t out = (int64_t)os.num, in = m_.values[xv].width;
            // names as gala.cu's: efc<k> attention vectors (FFN_OP_EDGE), sfc<k> a second
            // FFN of the layer input (FFN_OP_SELF), fc<k> otherwise
            const char *prefix = out == 1 ? "efc" : (xv == c.in_feats && ffn_reads_input_twice(c) ? "sfc" : "fc");
            if (c.heads > 1 && out == 1) {
                // one attention vector per head over that head's slice of x
                if (in % c.heads != 0)
                    throw DslError(e.at, "gat_heads(" + std::to_string(c.heads) + "): attention input of " +
                                             std::to_string(in) + " columns is not a whole number of heads");
                const int w = new_weight(prefix, in, 1);
                m_.weights[w].heads = c.heads;
                return Sym::of_val(node(Op::Ffn, {xv}, "attn", Kind::Node, c.heads, c, 0, w));
            }
            const int64_t width = out == 1 ? 1 : out * c.heads;  // H heads of `out` features
            const int w = new_weight(prefix, in, width);
            return Sym::of_val(node(Op::Ffn, {xv}, out == 1 ? "attn" : "res", Kind::Node, width, c, 0, w));
        }
        if (cp == "dsl.nn.scalar") {
            const Expr *x = arg(e, 0);
            if (!x || x->kind != Expr::Number) throw DslError(e.at, "scalar(initial value)");
            Sym s;
            s.t = Sym::Scalar;
            s.num = x->num;
            return s;
        }
        if (cp == "dsl.fn.softmax") {
            const Expr *x = arg(e, 1);
            if (!x) throw DslError(e.at, "softmax(G, edge_values)");
            const int xv = as_val(eval(*x, c), *x, "softmax");
            if (m_.values[xv].kind != Kind::Edge) throw DslError(x->at, "softmax needs edge values");
            return Sym::of_val(node(Op::Softmax, {xv}, "attn", Kind::Edge, m_.values[xv].width, c));
        }
        if (cp == "dsl.non_ln.ReLU" || cp == "dsl.non_ln.LeakyReLU") {
            const Expr *x = arg(e, 0);
            if (!x) throw DslError(e.at, "non-linearity needs an argument");
            const int xv = as_val(eval(*x, c), *x, "non-linearity");
            return apply_nonln(cp == "dsl.non_ln.ReLU" ? 1 : 2, xv, c);
        }
        // parameters bound to functions
        auto it = e.obj && e.obj->kind == Expr::Ident ? c.env.find(e.obj->name) : c.env.end();
        if (it != c.env.end()) {
            const Sym &f = it->second;
            if (f.t == Sym::NonLn) {
                const Expr *x = arg(e, 0);
                if (!x) throw DslError(e.at, "non-linearity needs an argument");
                return apply_nonln(f.nonln, as_val(eval(*x, c), *x, "non-linearity"), c);
            }
            if (f.t == Sym::AggrFn) {
                const Expr *g = arg(e, 0), *x = arg(e, 1);
                if (!g || !x) throw DslError(e.at, "aggregate_fn(G.graphs, x)");
                const int xv = as_val(eval(*x, c), *x, "aggregate");
                if (m_.values[xv].kind != Kind::Node) throw DslError(x->at, "aggregate needs node features");
                std::vector<int> in{xv};
                if (c.edge_vals >= 0) in.push_back(c.edge_vals);
                int out = node(Op::Aggregate, in, "res", Kind::Node, m_.values[xv].width, c);
                if (f.s == "mul_mean") {
                    // mean = deg^-1 * sum: SAGE_OPS' DEGREES, POWER(normalization_value
                    // = -1), AGGREGATE, MULT_NORM_RES (frontend.y:160-168, metadata :73)
                    const int deg = graph_value(Op::Degrees, 0, -1, c);
                    const int inv = graph_value(Op::Power, -1.0, deg, c);
                    out = node(Op::RowBroadcast, {inv, out}, "res_n", Kind::Node,
                               m_.values[out].width, c);
                }
                return Sym::of_val(out);
            }
            if (f.t == Sym::EdgeFn) {
                const Expr *a = arg(e, 1), *b = arg(e, 2);
                if (!a || !b) throw DslError(e.at, "edge_fn(G, a_src, a_dst)");
                const int av = as_val(eval(*a, c), *a, "edge_fn"), bv = as_val(eval(*b, c), *b, "edge_fn");
                const int64_t h = m_.values[av].width;
                if (m_.values[bv].width != h) throw DslError(e.at, "edge_fn: source / destination logits differ in heads");
                const int s = node(Op::EdgeAdd, {av, bv}, "attn", Kind::Edge, h, c);
                // ATTN -> addLeakyReLU(0.2) (frontend.y:1000-1003, 786-800)
                return Sym::of_val(node(Op::LeakyRelu, {s}, "attn", Kind::Edge, h, c, 0.2));
            }
        }
        throw DslError(e.at, "unknown function '" + (cp.empty() ? std::string("?") : cp) + "'");
    }

    // SAGE's self FFN: the layer body reads its input features in two FFNs
    bool ffn_reads_input_twice(const LayerCtx &c) const {
        for (const Node &n : m_.nodes)
            if (n.layer == c.layer && n.op == Op::Ffn && !n.in.empty() && n.in[0] != c.in_feats)
                return true;
        return false;
    }

    Sym apply_nonln(int kind, int xv, LayerCtx &c) {
        if (kind == 0) return Sym::of_val(xv);  // null: identity (nonln_present = false)
        if (kind == 1)
            return Sym::of_val(node(Op::Relu, {xv}, "res", m_.values[xv].kind, m_.values[xv].width, c));
        return Sym::of_val(node(Op::LeakyRelu, {xv}, "res", m_.values[xv].kind,
                                m_.values[xv].width, c, 0.2));
    }
};

}  // namespace

Module lower(const Program &prog) { return Lowering(prog).run(); }

}  // namespace galac
