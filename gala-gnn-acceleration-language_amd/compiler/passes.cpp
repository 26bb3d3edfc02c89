// passes.cpp — galac's middle-end.
//
// The reference's GALATransformations (src/middle-end/middle-end.h) rewrite CIR node
// lists by swapping neighbours and renaming data nodes.  The same decisions are made
// here on SSA use-def chains:
//   operator reordering   complexityOperatorReordering (middle-end.h:494-876): an FFN
//                         that shrinks the feature width moves before the aggregation /
//                         row-broadcast / eps-scale chain feeding it, one that widens
//                         moves after the chain it feeds (aggregate at the narrow width)
//   sparse rewrite        sparsityAwareRewrites (:213-407): norm * A (norm * x) on an
//                         is_sparser graph -> A_w x with w_e = norm_row * norm_col
//                         computed once (AGGREGATE_EDGE_MUL)
//   code motion           trainingInvariantCodeMotion (:409-492): FFNs move after the
//                         aggregations they feed so the aggregation of the input
//                         features becomes training-invariant, then every invariant
//                         node is computed once, before the loop
//   training subgraph     trainingSubGraph (:39-211): aggregation c of L reads the c-th
//                         mask subgraph (graph 1 + c)
// and, MI355X-specific (no reference counterpart):
//   fusion                ROW_BROADCAST / AGGREGATE / ROW_BROADCAST -> one GcnAggregate
//                         (prescale pass + dst-scaled SpMM); AGGREGATE_EDGE_SUM /
//                         LEAKY_RELU / SOFTMAX / attention AGGREGATE -> one GatAggregate
//                         (gala_gat_fwd_f32).  Both keep the reference's roundings.
#include <algorithm>
#include <functional>
#include <set>

#include "ir.h"

namespace galac {

namespace {

bool linear_unary(const Module &m, const Node &n) {
    // ops f with f(x W + b) handled like the reference: RowBroadcast (x is in[1]),
    // Aggregate (x is in[0]; any edge weights are fixed within a forward), ScaleEps
    if (n.dead) return false;
    // per-head attention weights (gat_heads) scale each head's columns differently: an FFN
    // that mixes heads does not commute with that aggregation
    if (n.op == Op::Aggregate && n.in.size() > 1 && m.values[n.in[1]].width > 1) return false;
    return n.op == Op::RowBroadcast || n.op == Op::Aggregate || n.op == Op::ScaleEps;
}

int data_input_index(const Node &n) { return n.op == Op::RowBroadcast ? 1 : 0; }

void set_width(Module &m, int value, int64_t w) { m.values[value].width = w; }

// Move node `a` (which must come before `b` in program order) directly after `b`.
void move_after(Module &m, int a, int b) {
    Node na = m.nodes[a];
    m.nodes.erase(m.nodes.begin() + a);
    if (b > a) --b;
    m.nodes.insert(m.nodes.begin() + b + 1, na);
}
void move_before(Module &m, int a, int b) {
    Node na = m.nodes[a];
    m.nodes.erase(m.nodes.begin() + a);
    if (b > a) --b;
    m.nodes.insert(m.nodes.begin() + b, na);
}

// FFN f = Ffn(y) with y = op(x) (single use) -> y' = Ffn(x), f' = op(y').  Returns true
// if it rewrote.  The FFN's output value keeps its id (its users are unchanged).
bool hoist_ffn_before(Module &m, int fi) {
    Node &f = m.nodes[fi];
    const int y = f.in[0];
    const int pi = m.producer(y);
    if (pi < 0 || m.uses(y).size() != 1) return false;
    Node &p = m.nodes[pi];
    if (!linear_unary(m, p) || p.hoisted != f.hoisted) return false;
    const int di = data_input_index(p);
    const int x = p.in[di];
    const int64_t out_w = m.values[f.out].width;
    // f now reads x and writes y (narrow); p reads y and writes f.out
    const int fout = f.out;
    f.in[0] = x;
    f.out = y;
    set_width(m, y, out_w);
    p.in[di] = y;
    p.out = fout;
    m.values[y].invariant = false;
    m.values[fout].invariant = false;
    move_before(m, fi, pi);  // keep program order: f before p
    return true;
}

// FFN f = Ffn(x) whose only user is op(f) -> op'(x), then Ffn.  Returns true if rewrote.
bool sink_ffn_after(Module &m, int fi, bool require_invariant_input) {
    Node &f = m.nodes[fi];
    const auto u = m.uses(f.out);
    if (u.size() != 1) return false;
    const int ui = u[0];
    Node &p = m.nodes[ui];
    if (!linear_unary(m, p) || p.in[data_input_index(p)] != f.out) return false;
    if (p.op == Op::ScaleEps) return false;  // keep the learned eps on the narrow side
    if (require_invariant_input) {
        if (!m.values[f.in[0]].invariant) return false;
        for (size_t k = 0; k < p.in.size(); ++k)
            if ((int)k != data_input_index(p) && !m.values[p.in[k]].invariant) return false;
    }
    const int x = f.in[0], fy = f.out, py = p.out;
    const int64_t in_w = m.values[x].width;
    // p now reads x and writes fy (wide), f reads fy and writes py
    p.in[data_input_index(p)] = x;
    p.out = fy;
    set_width(m, fy, in_w);
    f.in[0] = fy;
    f.out = py;
    move_after(m, fi, ui);
    return true;
}

void recompute_invariance(Module &m, bool dynamic_sampling) {
    for (Node &n : m.nodes) {
        if (n.dead) continue;
        bool inv = n.weight < 0 && n.op != Op::ScaleEps;
        if (n.op == Op::Input || n.op == Op::Degrees || n.op == Op::SampledDegrees) inv = true;
        if (dynamic_sampling && (n.op == Op::Aggregate || n.op == Op::GcnAggregate)) inv = false;
        for (int v : n.in)
            if (v >= 0) inv = inv && m.values[v].invariant;
        m.values[n.out].invariant = inv;
    }
}

void reorder(Module &m) {
    bool changed = true;
    int guard = 0;
    while (changed && guard++ < 1000) {
        changed = false;
        for (int i = 0; i < (int)m.nodes.size() && !changed; ++i) {
            const Node &f = m.nodes[i];
            if (f.dead || f.op != Op::Ffn) continue;
            const Weight &w = m.weights[f.weight];
            if (w.out < w.in) changed = hoist_ffn_before(m, i);
            else if (w.out > w.in) changed = sink_ffn_after(m, i, false);
            if (changed)
                m.notes.push_back("reorder: " + w.name + " (" + std::to_string(w.in) + "->" +
                                  std::to_string(w.out) + ") moved " +
                                  (w.out < w.in ? "before" : "after") + " a " +
                                  "row-broadcast/aggregation");
        }
    }
}

void sparse_rewrite(Module &m) {
    for (int i = 0; i < (int)m.nodes.size(); ++i) {
        Node &agg = m.nodes[i];
        if (agg.dead || agg.op != Op::Aggregate || agg.in.size() != 1) continue;
        const int pre = m.producer(agg.in[0]);
        const auto post_u = m.uses(agg.out);
        if (pre < 0 || post_u.size() != 1 || m.uses(agg.in[0]).size() != 1) continue;
        Node &rb1 = m.nodes[pre];
        Node &rb2 = m.nodes[post_u[0]];
        if (rb1.op != Op::RowBroadcast || rb2.op != Op::RowBroadcast || rb2.in[1] != agg.out)
            continue;
        // w = norm1[row] * norm2[col] once (aggregate_edge_mul); norm * A (norm * x) =
        // A_w x with the row norm on the left (middle-end.h:249-300)
        int w = -1;
        for (const Node &n : m.nodes)
            if (!n.dead && n.op == Op::EdgeMul && n.in[0] == rb2.in[0] && n.in[1] == rb1.in[0])
                w = n.out;
        if (w < 0) {
            w = m.add_value("val", Kind::Edge, 1, true);
            Node em{Op::EdgeMul};
            em.in = {rb2.in[0], rb1.in[0]};
            em.out = w;
            m.nodes.insert(m.nodes.begin() + pre, em);
            ++i;
        }
        Node &a2 = m.nodes[i];
        Node &r1 = m.nodes[m.producer(a2.in[0])];
        Node &r2 = m.nodes[m.uses(a2.out)[0]];
        const int x = r1.in[1], out = r2.out;
        r1.dead = true;
        r2.dead = true;
        a2.in = {x, w};
        a2.out = out;
        m.notes.push_back("sparse rewrite: norm * A (norm * x) -> A_w x, w = norm_i * norm_j");
    }
}

void code_motion(Module &m, bool dynamic_sampling) {
    // sink FFNs past the linear ops they feed while their input is invariant (the
    // enableTim reordering, middle-end.h:411-416, 521-606)
    recompute_invariance(m, dynamic_sampling);
    bool changed = true;
    int guard = 0;
    while (changed && guard++ < 1000) {
        changed = false;
        for (int i = 0; i < (int)m.nodes.size() && !changed; ++i) {
            const Node &f = m.nodes[i];
            if (f.dead || f.op != Op::Ffn) continue;
            const std::string wn = m.weights[f.weight].name;
            changed = sink_ffn_after(m, i, true);
            if (changed) {
                recompute_invariance(m, dynamic_sampling);
                m.notes.push_back("code motion: " + wn +
                                  " moved after an invariant aggregation/row-broadcast");
            }
        }
    }
    recompute_invariance(m, dynamic_sampling);
    int hoisted = 0;
    for (Node &n : m.nodes)
        if (!n.dead && m.values[n.out].invariant && !n.hoisted) {
            n.hoisted = true;
            if (n.op != Op::Input) ++hoisted;
        }
    if (hoisted)
        m.notes.push_back("code motion: " + std::to_string(hoisted) +
                          " training-invariant op(s) computed once before the loop");
}

void graph_only_hoist(Module &m) {
    // without code motion the reference recomputes degrees every forward
    // (gala_inference); still hoist nothing but the input itself
    for (Node &n : m.nodes) n.hoisted = n.op == Op::Input;
}

bool is_aggregate(Op op) {
    return op == Op::Aggregate || op == Op::GcnAggregate || op == Op::GatAggregate;
}

void subgraphs(Module &m) {
    int c = 0;
    for (Node &n : m.nodes)
        if (!n.dead && is_aggregate(n.op)) n.graph = 1 + c++;
    m.num_graphs = 1 + c;
    // edge ops feeding an aggregation live on its graph's edge list
    for (Node &n : m.nodes) {
        if (n.dead || !is_aggregate(n.op) || n.in.size() < 2) continue;
        std::function<void(int)> mark = [&](int v) {
            const int p = m.producer(v);
            if (p < 0) return;
            Node &pn = m.nodes[p];
            if (m.values[pn.out].kind != Kind::Edge) return;
            pn.graph = n.graph;
            for (int w : pn.in)
                if (w >= 0) mark(w);
        };
        mark(n.in[1]);
    }
    if (c) m.notes.push_back("training subgraph: " + std::to_string(c) + " aggregation(s) on mask subgraphs");
}

void fuse(Module &m) {
    // GAT: Softmax(LeakyRelu(EdgeAdd(aL, aR))) feeding only an attention Aggregate
    for (int i = 0; i < (int)m.nodes.size(); ++i) {
        Node &agg = m.nodes[i];
        if (agg.dead || agg.op != Op::Aggregate || agg.in.size() != 2) continue;
        const int si = m.producer(agg.in[1]);
        if (si < 0 || m.nodes[si].op != Op::Softmax || m.uses(agg.in[1]).size() != 1) continue;
        const int li = m.producer(m.nodes[si].in[0]);
        if (li < 0 || m.nodes[li].op != Op::LeakyRelu || m.uses(m.nodes[si].in[0]).size() != 1) continue;
        const int ei = m.producer(m.nodes[li].in[0]);
        if (ei < 0 || m.nodes[ei].op != Op::EdgeAdd || m.uses(m.nodes[li].in[0]).size() != 1) continue;
        agg.op = Op::GatAggregate;
        agg.param = m.nodes[li].param;
        agg.in = {m.nodes[ei].in[0], m.nodes[ei].in[1], agg.in[0]};
        m.nodes[si].dead = m.nodes[li].dead = m.nodes[ei].dead = true;
        m.notes.push_back("fuse: edge add + leaky relu + softmax + aggregation -> gat_aggregate");
        // attnR = ffn(res, out=1) of the aggregated res itself: the kernels recompute the
        // source logit from the X row they gather (gat_aggregate_ffn), no aR[col] reads
        const int fi = m.producer(agg.in[1]);
        if (fi >= 0 && m.nodes[fi].op == Op::Ffn && m.nodes[fi].weight >= 0 &&
            m.nodes[fi].in[0] == agg.in[2] && m.weights[m.nodes[fi].weight].out == 1 &&
            m.uses(agg.in[1]).size() == 1 && m.nodes[fi].hoisted == agg.hoisted) {
            agg.weight = m.nodes[fi].weight;
            agg.in[1] = -1;
            m.nodes[fi].dead = true;
            m.notes.push_back("fuse: attention linear of the aggregated rows recomputed in the "
                              "GAT kernels -> gat_aggregate_ffn");
        }
    }
    // GCN: [RowBroadcast(pre)] -> Aggregate (unweighted or fixed weights) -> [RowBroadcast(post)]
    for (int i = 0; i < (int)m.nodes.size(); ++i) {
        Node &agg = m.nodes[i];
        if (agg.dead || agg.op != Op::Aggregate) continue;
        if (agg.in.size() == 2) continue;  // attention weights: separate autograd op
        int x = agg.in[0], pre = -1, post = -1, out = agg.out;
        const int pi = m.producer(x);
        if (pi >= 0 && m.nodes[pi].op == Op::RowBroadcast && m.uses(x).size() == 1 &&
            m.nodes[pi].hoisted == agg.hoisted) {
            pre = m.nodes[pi].in[0];
            x = m.nodes[pi].in[1];
            m.nodes[pi].dead = true;
        }
        const auto u = m.uses(agg.out);
        if (u.size() == 1 && m.nodes[u[0]].op == Op::RowBroadcast && m.nodes[u[0]].in[1] == agg.out &&
            m.nodes[u[0]].hoisted == agg.hoisted && agg.out != m.output) {
            post = m.nodes[u[0]].in[0];
            out = m.nodes[u[0]].out;
            m.nodes[u[0]].dead = true;
        }
        agg.op = Op::GcnAggregate;
        agg.in = {x, pre, post};
        agg.out = out;
        if (pre >= 0 || post >= 0)
            m.notes.push_back(std::string("fuse: ") + (pre >= 0 ? "row-broadcast + " : "") +
                              "aggregation" + (post >= 0 ? " + row-broadcast" : "") +
                              " -> gcn_aggregate");
    }
    // GCN prologue: relu([act *] z) feeding only a GcnAggregate's (pre-scaled) input becomes
    // one elementwise pass in front of the SpMM (pre * relu(act * z)); act must be a
    // graph-invariant row vector (the layer's norm) -- its gradient is never needed
    for (int i = 0; i < (int)m.nodes.size(); ++i) {
        Node &agg = m.nodes[i];
        if (agg.dead || agg.op != Op::GcnAggregate || agg.param != 0) continue;
        const int x = agg.in[0];
        const int ri = m.producer(x);
        if (ri < 0 || m.nodes[ri].op != Op::Relu || m.uses(x).size() != 1 ||
            m.nodes[ri].hoisted != agg.hoisted)
            continue;
        int z = m.nodes[ri].in[0], act = -1;
        const int bi = m.producer(z);
        if (bi >= 0 && m.nodes[bi].op == Op::RowBroadcast && m.uses(z).size() == 1 &&
            m.nodes[bi].hoisted == agg.hoisted && m.values[m.nodes[bi].in[0]].invariant) {
            act = m.nodes[bi].in[0];
            z = m.nodes[bi].in[1];
            m.nodes[bi].dead = true;
        }
        m.nodes[ri].dead = true;
        agg.in = {z, agg.in[1], agg.in[2], act};
        agg.param = 1;
        m.notes.push_back(std::string("fuse: ") + (act >= 0 ? "row-broadcast + " : "") +
                          "relu in front of gcn_aggregate -> one elementwise pass");
    }
    // keep program order valid: a fused node must come after its inputs' producers
    for (int i = 0; i < (int)m.nodes.size(); ++i) {
        if (m.nodes[i].dead) continue;
        for (int v : m.nodes[i].in) {
            if (v < 0) continue;
            const int p = m.producer(v);
            if (p > i) {
                move_after(m, i, p);
                i = -1;
                break;
            }
        }
    }
}

void dce(Module &m) {
    bool changed = true;
    while (changed) {
        changed = false;
        for (Node &n : m.nodes) {
            if (n.dead || n.op == Op::Input || n.out == m.output) continue;
            if (m.uses(n.out).empty()) {
                n.dead = true;
                changed = true;
            }
        }
    }
    m.nodes.erase(std::remove_if(m.nodes.begin(), m.nodes.end(), [](const Node &n) { return n.dead; }),
                  m.nodes.end());
    // drop weights no node uses any more, keeping their order
    std::vector<int> remap(m.weights.size(), -1);
    std::vector<Weight> kept;
    for (const Node &n : m.nodes)
        if (n.weight >= 0 && remap[n.weight] < 0) {
            remap[n.weight] = 0;
        }
    for (size_t k = 0; k < m.weights.size(); ++k)
        if (remap[k] == 0) {
            remap[k] = (int)kept.size();
            kept.push_back(m.weights[k]);
        }
    for (Node &n : m.nodes)
        if (n.weight >= 0) n.weight = remap[n.weight];
    m.weights = kept;
}

}  // namespace

void run_passes(Module &m, bool fusion) {
    Schedule &s = m.sched;
    const bool dyn = s.kernel_sample > 0 && s.dynamic_sample;
    if (s.operator_reordering) reorder(m);
    if (s.sparse_rewrites && s.sparse) sparse_rewrite(m);
    dce(m);
    if (s.train_code_motion) code_motion(m, dyn);
    else graph_only_hoist(m);
    if (fusion) fuse(m);
    dce(m);
    if (s.training_subgraph) {
        if (s.print_accuracy)
            m.notes.push_back("training subgraph skipped: print_accuracy evaluates test rows, "
                              "which the train-mask subgraphs leave out");
        else if (s.kernel_sample > 0 || s.data_sample > 0)
            m.notes.push_back("training subgraph skipped: sampled aggregation");
        else if (std::any_of(m.nodes.begin(), m.nodes.end(), [](const Node &n) {
                     return n.op == Op::GatAggregate || (n.op == Op::Aggregate && n.in.size() > 1);
                 }))
            m.notes.push_back("training subgraph skipped: edge-weighted aggregation (its "
                              "backward on the transposed subgraph would need permuted weights)");
        else
            subgraphs(m);
    }
}

}  // namespace galac
