// host_sanitize.cpp -- the host libraries' code under AddressSanitizer + UBSan (test
// infrastructure; tests/test_host_sanitizers_cpu.py builds and runs it).
//
// csrc/host_graph.cpp (the gala_host_* graph builders of libgala_hip.so) and
// csrc/cpu_backend.cpp (libgala_cpu.so, the host twin of every operator) are compiled
// together with this driver, -fsanitize=address,undefined, and every builder and operator
// runs on seeded random graphs with the corners the GPU kernels handle: empty graphs, empty
// rows, one hub row, column-tiled segments, kernel sampling, padded strides, 1..8 heads,
// the GCN epilogue.  Buffers are allocated exactly to the sizes the ABI documents, so an
// out-of-bounds read or write in either library aborts the run.  The SpMM is also compared
// with a plain loop (the CSR-order sum), so the harness checks something beyond memory.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "gala_cpu.h"

namespace {

#define CHECK(x)                                                                      \
    do {                                                                              \
        int s_ = (x);                                                                 \
        if (s_ != GALA_OK) {                                                          \
            fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, s_);          \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

struct Graph {
    int64_t n = 0, nnz = 0;
    std::vector<int32_t> rowptr, col;
};

Graph random_graph(std::mt19937 &rng, int64_t n, double mean_deg, bool empty_rows, bool hub) {
    std::vector<int32_t> src, dst;
    std::uniform_int_distribution<int64_t> pick(0, n > 0 ? n - 1 : 0);
    const int64_t m = n > 0 ? (int64_t)(mean_deg * n) : 0;
    for (int64_t i = 0; i < m; ++i) {
        int64_t s = pick(rng);
        if (empty_rows) s %= (n / 3 > 0 ? n / 3 : 1);
        src.push_back((int32_t)s);
        dst.push_back((int32_t)pick(rng));
    }
    if (hub && n > 0) {
        const int32_t h = (int32_t)pick(rng);
        for (int i = 0; i < 3000; ++i) {
            src.push_back(h);
            dst.push_back((int32_t)pick(rng));
        }
    }
    Graph g;
    g.n = n;
    g.nnz = (int64_t)src.size();
    g.rowptr.assign(n + 1, 0);
    g.col.assign(g.nnz, 0);
    std::vector<int32_t> perm(g.nnz);
    CHECK(gala_host_csr_build(n, n, g.nnz, src.data(), dst.data(), g.rowptr.data(), g.col.data(), perm.data()));
    return g;
}

gala_csr_t view(const Graph &g, const float *val = nullptr, int32_t heads = 1) {
    gala_csr_t A;
    memset(&A, 0, sizeof(A));
    A.n_rows = g.n;
    A.n_cols = g.n;
    A.nnz = g.nnz;
    A.rowptr = g.rowptr.data();
    A.col = g.col.data();
    A.val = val;
    A.val_heads = heads;
    A.n_seg = 1;
    return A;
}

std::vector<float> uniform(std::mt19937 &rng, size_t n, float lo = -1.0f, float hi = 1.0f) {
    std::uniform_real_distribution<float> d(lo, hi);
    std::vector<float> v(n);
    for (auto &x : v) x = d(rng);
    return v;
}

void check_spmm(const Graph &g, const std::vector<float> &X, int64_t ldx, const std::vector<float> &Y, int64_t ldy,
                int F) {
    for (int64_t r = 0; r < g.n; ++r)
        for (int f = 0; f < F; ++f) {
            float acc = 0.0f;
            for (int32_t e = g.rowptr[r]; e < g.rowptr[r + 1]; ++e) acc = acc + X[(size_t)g.col[e] * ldx + f];
            if (memcmp(&acc, &Y[(size_t)r * ldy + f], sizeof(float)) != 0) {
                fprintf(stderr, "spmm mismatch row %lld f %d\n", (long long)r, f);
                exit(1);
            }
        }
}

void one_case(std::mt19937 &rng, int it) {
    const int64_t n = it == 0 ? 0 : (int64_t)(rng() % 700) + 1;
    const Graph g = random_graph(rng, n, (double)(rng() % 12), rng() % 3 == 0, rng() % 3 == 0);
    const int heads = 1 << (rng() % 4);
    const int D = 1 + (int)(rng() % 8);
    const int F = heads * D;
    const int64_t ld = F + (int64_t)(rng() % 5);  // padded stride
    const auto X = uniform(rng, (size_t)std::max<int64_t>(n, 1) * ld);
    gala_csr_t A = view(g);

    // SpMM (plain, weighted, sampled, accumulate), checked against the CSR-order sum
    std::vector<float> Y((size_t)std::max<int64_t>(n, 1) * ld, 0.0f);
    CHECK(gala_cpu_spmm_f32(&A, X.data(), ld, Y.data(), ld, F, nullptr, nullptr, 0, 0, 0, 0, nullptr));
    check_spmm(g, X, ld, Y, ld, F);
    const auto w = uniform(rng, (size_t)std::max<int64_t>(g.nnz, 1) * heads, 0.0f, 1.0f);
    gala_csr_t Aw = view(g, w.data(), heads);
    CHECK(gala_cpu_spmm_f32(&Aw, X.data(), ld, Y.data(), ld, F, nullptr, nullptr, GALA_SPMM_ACCUM, 0, 0, 0,
                            nullptr));
    const auto s = uniform(rng, (size_t)std::max<int64_t>(n, 1));
    CHECK(gala_cpu_spmm_f32(&A, X.data(), ld, Y.data(), ld, F, s.data(), s.data(), 0, 0, 0, 0, nullptr));
    CHECK(gala_cpu_spmm_f32(&A, X.data(), ld, Y.data(), ld, F, nullptr, nullptr, GALA_SPMM_SAMPLE, 5, 5, 7,
                            nullptr));
    // the GCN epilogue: deg norm from the rowptr, the next input beside the output
    std::vector<float> Y2((size_t)std::max<int64_t>(n, 1) * ld, 0.0f);
    gala_spmm_epilogue_t epi;
    memset(&epi, 0, sizeof(epi));
    epi.dst_deg_rsqrt = 1;
    epi.Y2 = Y2.data();
    epi.ldy2 = ld;
    CHECK(gala_cpu_spmm_ex_f32(&A, X.data(), ld, Y.data(), ld, F, nullptr, nullptr, 0, 0, 0, 0, &epi, nullptr));
    CHECK(gala_cpu_row_broadcast_deg_f32(&A, F, X.data(), ld, Y2.data(), ld, nullptr));
    std::vector<float> deg((size_t)std::max<int64_t>(n, 1));
    CHECK(gala_cpu_degree_f32(&A, deg.data(), -0.5f, 0, 0, nullptr));

    // column-tiled segments
    if (n > 1) {
        const int64_t cpp = 1 + (int64_t)(rng() % n);
        std::vector<int32_t> bp(n + 2);
        const int64_t nb = gala_host_col_breakpoints(n, cpp, bp.data(), (int64_t)bp.size());
        if (nb < 2) exit(1);
        const int32_t nseg = (int32_t)(nb - 1);
        std::vector<int32_t> trp((size_t)(n + 1) * nseg), tcol(std::max<int64_t>(g.nnz, 1)), bounds(2 * nseg);
        CHECK(gala_host_col_tile(n, g.rowptr.data(), g.col.data(), nullptr, nseg, bp.data(), trp.data(), tcol.data(),
                                 nullptr, bounds.data()));
        gala_csr_t T = view(g);
        T.rowptr = trp.data();
        T.col = tcol.data();
        T.n_seg = nseg;
        T.seg_bounds = bounds.data();
        CHECK(gala_cpu_spmm_f32(&T, X.data(), ld, Y.data(), ld, F, nullptr, nullptr, 0, 0, 0, 0, nullptr));
        check_spmm(g, X, ld, Y, ld, F);  // segments summed in order: the same sums
    }
    // kernel-sampled layout (rows with edges only)
    bool all_rows = n > 0;
    for (int64_t r = 0; r < n; ++r) all_rows = all_rows && g.rowptr[r + 1] > g.rowptr[r];
    if (all_rows) {
        const int ns = 1 + (int)(rng() % 6);
        std::vector<int32_t> srp(n + 1), scol((size_t)n * ns);
        CHECK(gala_host_sample_ab(n, g.rowptr.data(), g.col.data(), nullptr, ns, 5, 7, srp.data(), scol.data(),
                                  nullptr));
    }
    // split plan, row order, transpose
    if (n > 0) {
        int64_t nrs = 0, nch = 0;
        CHECK(gala_host_split_plan(n, g.rowptr.data(), 64, 32, nullptr, nullptr, nullptr, &nrs, &nch));
        std::vector<int32_t> rows(std::max<int64_t>(nrs, 1)), rc0(nrs + 1), crow(std::max<int64_t>(nch, 1));
        CHECK(gala_host_split_plan(n, g.rowptr.data(), 64, 32, rows.data(), rc0.data(), crow.data(), &nrs, &nch));
        std::vector<int32_t> order(n);
        CHECK(gala_host_row_order(n, g.rowptr.data(), order.data()));
        std::vector<int32_t> tr(n + 1), tc(std::max<int64_t>(g.nnz, 1)), tp(std::max<int64_t>(g.nnz, 1));
        CHECK(gala_host_csr_transpose(n, n, g.rowptr.data(), g.col.data(), tr.data(), tc.data(), tp.data()));
    }
    if (g.nnz == 0) return;

    // edge operators, exact-size per-edge buffers
    const size_t E = (size_t)g.nnz, EH = E * heads, NH = (size_t)n * heads;
    const auto aL = uniform(rng, NH), aR = uniform(rng, NH);
    std::vector<float> ev(EH), ev2(EH), rowv(NH);
    CHECK(gala_cpu_sddvv_f32(&A, aL.data(), aR.data(), heads, GALA_SDDVV_ADD_LRELU, 0.2f, ev.data(), nullptr));
    CHECK(gala_cpu_row_sum_f32(&A, ev.data(), heads, 1e-12f, rowv.data(), 0, nullptr));
    CHECK(gala_cpu_row_scale_f32(&A, rowv.data(), heads, ev.data(), nullptr));
    CHECK(gala_cpu_sddmm_dot_f32(&A, X.data(), ld, X.data(), ld, F, heads, ev2.data(), nullptr));
    for (int mode : {GALA_SOFTMAX_REF, GALA_SOFTMAX_FIXED}) {
        CHECK(gala_cpu_edge_softmax_fwd_f32(&A, ev2.data(), heads, mode, ev.data(), nullptr));
        CHECK(gala_cpu_edge_softmax_bwd_f32(&A, ev.data(), ev2.data(), heads, mode, ev2.data(), nullptr));
        std::vector<float> alpha(EH), dlog(EH), daL(NH);
        CHECK(gala_cpu_gat_fwd_f32(&A, aL.data(), aR.data(), X.data(), ld, F, heads, 0.2f, mode, Y.data(), ld,
                                   alpha.data(), nullptr));
        CHECK(gala_cpu_gat_bwd_f32(&A, aL.data(), aR.data(), X.data(), ld, X.data(), ld, F, heads, 0.2f, mode,
                                   alpha.data(), dlog.data(), daL.data(), nullptr));
    }
    // REF row statistics pair, the source logit recomputed from X, p parked
    const auto wR = uniform(rng, F), bR = uniform(rng, heads);
    std::vector<float> Ys((size_t)n * ld), Ym((size_t)n * ld), q(NH), sma(NH), aRo(NH), p(EH), dX((size_t)n * ld),
        daL(NH);
    CHECK(gala_cpu_gat_fwd_stats_f32(&A, aL.data(), nullptr, wR.data(), bR.data(), X.data(), ld, F, heads, 0.2f,
                                     Ys.data(), ld, q.data(), Ym.data(), ld, sma.data(), aRo.data(), p.data(),
                                     nullptr));
    CHECK(gala_cpu_gat_bwd_stats_f32(&A, aL.data(), aRo.data(), nullptr, X.data(), ld, F, heads, 0.2f, q.data(),
                                     Ys.data(), ld, Ym.data(), ld, sma.data(), dX.data(), ld, daL.data(), nullptr));
    CHECK(gala_cpu_gat_bwd_stats_f32(&A, aL.data(), nullptr, p.data(), X.data(), ld, F, heads, 0.2f, q.data(),
                                     Ys.data(), ld, Ym.data(), ld, sma.data(), dX.data(), ld, daL.data(), nullptr));
    CHECK(gala_cpu_gat_bwd_fused_f32(&A, aL.data(), aRo.data(), nullptr, nullptr, X.data(), ld, X.data(), ld, F,
                                     heads, 0.2f, q.data(), dX.data(), ld, daL.data(), nullptr));
    std::vector<float> U((size_t)n * ld), sums(NH), Um((size_t)n * ld), msums(NH);
    CHECK(gala_cpu_gat_fwd_partial_stats_f32(&A, aL.data(), aR.data(), nullptr, nullptr, X.data(), ld, F, heads,
                                             0.2f, U.data(), ld, sums.data(), Um.data(), ld, msums.data(), nullptr));
    std::vector<float> ha(NH), hdx((size_t)n * ld);
    CHECK(gala_cpu_head_attn_f32(n, F, heads, X.data(), ld, wR.data(), bR.data(), ha.data(), nullptr));
    CHECK(gala_cpu_head_attn_bwd_f32(n, F, heads, ha.data(), wR.data(), hdx.data(), ld, 1, nullptr));
    // FFN forward and the weight gradients
    const int M = 1 + (int)(rng() % 9);
    const auto W = uniform(rng, (size_t)M * F), b = uniform(rng, M);
    std::vector<float> Z((size_t)n * M), dW((size_t)M * F), db(M);
    CHECK(gala_cpu_ffn_fwd_f32(n, F, M, X.data(), ld, W.data(), b.data(), Z.data(), M, nullptr));
    const int64_t wsb = gala_cpu_dense_grad_workspace(n, F, M);
    std::vector<char> ws((size_t)std::max<int64_t>(wsb, 1));
    CHECK(gala_cpu_dense_grad_f32(n, F, M, X.data(), ld, Z.data(), M, dW.data(), db.data(), 0, ws.data(), wsb,
                                  nullptr));
}

}  // namespace

int main(int argc, char **argv) {
    const int cases = argc > 1 ? atoi(argv[1]) : 60;
    std::mt19937 rng(12345);
    for (int it = 0; it < cases; ++it) one_case(rng, it);
    printf("host sanitize: %d cases ok\n", cases);
    return 0;
}
