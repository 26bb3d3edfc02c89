// Edge-parallel ops of the GAT pipeline for gfx950: SDDVV (add / mul / add+LeakyReLU),
// edge->row sum, row->edge scale, SDDMM dot, edge-softmax forward/backward, the fused
// GAT aggregation and the edge-value permutation.
//
// Replaces the emitted kernels default_function_kernel_sddvv_{plus,mult}_undir
// (src/codegen/cuda.h:679-698, 848-867), spmm_backward_sddmm_32_{nln,eaggr}
// (505-524, 659-678), {softmax,mult}_sddvv_undir (525-562), sddmm_mult_undir_shared
// (699-734) and the torch compositions around them (src/codegen/common.h:735-810).
//
// Row-segment ops ("RS" kernels): a group of G lanes owns one row and strides over its
// edges (coalesced edge arrays), reductions use xor butterflies inside the group.
#include <stddef.h>

#include <algorithm>

#include "gala_internal.h"

namespace gala {

struct EdgeParams {
    const int32_t *rowptr;
    const int32_t *col;
    int64_t n_rows;
    int32_t heads;
    int32_t xcd_order;  // 1: XCD-aware block order (gala_internal.h); 0 on skewed graphs
    SegTable seg;
};

__device__ __forceinline__ void row_range(const EdgeParams &p, int s, int64_t row, int64_t &e0,
                                          int64_t &e1) {
    // EdgeParams is every edge kernel's first argument: read the table from kernarg
    KernargSegPtr seg = kernarg_segtable(offsetof(EdgeParams, seg));
    const int32_t *rp = p.rowptr + (int64_t)seg->rp[s] * (p.n_rows + 1);
    e0 = (int64_t)seg->base[s] + rp[row];
    e1 = (int64_t)seg->base[s] + rp[row + 1];
}

#define GALA_ROW_PROLOGUE(G)                                                          \
    const int lane = threadIdx.x & (kWave - 1);                                       \
    const int gl = lane & ((G)-1);                                                    \
    const int64_t blk_ = p.xcd_order ? logical_block_runs(blockIdx.x, gridDim.x, kXcdRun) \
                                     : (int64_t)blockIdx.x;                           \
    const int64_t row = (blk_ * (kBlock / kWave) + threadIdx.x / kWave)              \
                            * (kWave / (G)) + lane / (G);                             \
    const bool row_ok = row < p.n_rows;

// Device view of the hub-row plan: rows longer than `threshold` are cut into chunks of
// `chunk` edges that separate row groups run in parallel; their per-chunk partial state
// goes to ws (ws_cols floats per chunk) and fix-up kernels combine it in chunk order.
struct HubSplit {
    const int32_t *rows, *row_chunk0, *chunk_row;
    float *ws;
    int64_t ws_cols, n_chunks, n_rows_split;
    int32_t chunk, threshold;
};

// chunk c of a hub row -> its row group (n_seg == 1: plain CSR offsets)
#define GALA_CHUNK_PROLOGUE(G)                                                                  \
    const int lane = threadIdx.x & (kWave - 1);                                                 \
    const int gl = lane & ((G)-1);                                                              \
    const int64_t c = ((int64_t)blockIdx.x * (kBlock / kWave) + threadIdx.x / kWave) * (kWave / (G)) \
                      + lane / (G);                                                             \
    if (c >= sp.n_chunks) return;                                                               \
    const int32_t ri = sp.chunk_row[c];                                                         \
    const int64_t row = sp.rows[ri];                                                            \
    const int64_t r0 = p.rowptr[row], r1 = p.rowptr[row + 1];                                   \
    const int64_t e0 = r0 + (c - sp.row_chunk0[ri]) * (int64_t)sp.chunk;                       \
    const int64_t e1 = (e0 + sp.chunk < r1) ? e0 + sp.chunk : r1;

// ---- row-segment edge ops over flattened (edge, head) elements ----------------------
// With HP heads (a power of two dividing G) the row's HP*deg edge values are contiguous,
// lane g always handles head g % HP, and per-head reductions run over the xor offsets
// G/2 .. HP.  Non-power-of-two head counts use the *_generic kernels further down.
//
// Register tiles: a row slice is walked in tiles of G*K values; lane g holds the values
// t0 + g + k*G (k < K), so every lane has K coalesced loads in flight before it uses any
// (one load per lane at a time left these kernels latency-bound: 0.5 TB/s at 8 heads).
// When a row fits one tile, the second pass of softmax fwd/bwd runs from the registers.
constexpr int kTileK = 8;

template <int G, int HP>
__device__ __forceinline__ float head_sum(float v) {
#pragma unroll
    for (int o = G / 2; o >= HP; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
template <int G, int HP>
__device__ __forceinline__ float head_max(float v) {
#pragma unroll
    for (int o = G / 2; o >= HP; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// v[k] = base[t0 + gl + k*G] for indices < n, `fill` elsewhere
template <int G, int K>
__device__ __forceinline__ void load_tile(const float *base, int64_t n, int64_t t0, int gl,
                                          float fill, float (&v)[K]) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int64_t t = t0 + gl + (int64_t)k * G;
        v[k] = t < n ? base[t] : fill;
    }
}

// Hub rows (skewed graphs, A->split): the main kernel skips rows longer than the plan's
// threshold; *_chunk kernels run their 512-edge chunks in separate row groups, and
// *_fixup kernels (one thread per (hub row, head)) combine the chunk partials in chunk
// order.  The partials live in the plan's workspace (2*HP floats per chunk).
__device__ __forceinline__ bool hub_row(const EdgeParams &p, int32_t thr, int64_t row) {
    return thr > 0 && p.rowptr[row + 1] - p.rowptr[row] > thr;
}

// out[e, h] = a[row, h] op b[col_e, h] for the edges [e0, e1) of `row`
template <int G, int HP, int OP>
__device__ __forceinline__ void sddvv_range(const EdgeParams &p, const float *a, const float *b,
                                            float slope, float *out, int64_t row, int64_t e0,
                                            int64_t e1, int gl) {
    constexpr int LH = __builtin_ctz(HP);
    constexpr int K = kTileK;
    const int h = gl & (HP - 1);
    const float av = a[row * HP + h];
    const int64_t n = (e1 - e0) << LH;
    for (int64_t t0 = 0; t0 < n; t0 += G * K) {
        int32_t c[K];
        float bv[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int64_t t = t0 + gl + (int64_t)k * G;
            c[k] = p.col[e0 + ((t < n ? t : 0) >> LH)];
        }
#pragma unroll
        for (int k = 0; k < K; ++k) bv[k] = b[((int64_t)c[k] << LH) + h];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int64_t t = t0 + gl + (int64_t)k * G;
            if (t >= n) continue;
            float r;
            if (OP == GALA_SDDVV_MUL) {
                r = __fmul_rn(av, bv[k]);
            } else {
                r = __fadd_rn(av, bv[k]);
                if (OP == GALA_SDDVV_ADD_LRELU) r = r > 0.0f ? r : __fmul_rn(r, slope);
            }
            out[(e0 << LH) + t] = r;
        }
    }
}

template <int G, int HP, int OP>
__global__ __launch_bounds__(kBlock) void k_sddvv(EdgeParams p, const float *a, const float *b,
                                                  float slope, float *out, int32_t thr) {
    GALA_ROW_PROLOGUE(G);
    if (!row_ok || hub_row(p, thr, row)) return;
    for (int s = 0; s < p.seg.n; ++s) {
        int64_t e0, e1;
        row_range(p, s, row, e0, e1);
        sddvv_range<G, HP, OP>(p, a, b, slope, out, row, e0, e1, gl);
    }
}

template <int G, int HP, int OP>
__global__ __launch_bounds__(kBlock) void k_sddvv_chunk(EdgeParams p, const float *a, const float *b,
                                                        float slope, float *out, HubSplit sp) {
    GALA_CHUNK_PROLOGUE(G);
    sddvv_range<G, HP, OP>(p, a, b, slope, out, row, e0, e1, gl);
}

// the lane's partial sum of the (edge, head) values [e0*HP, e1*HP)
template <int G, int HP>
__device__ __forceinline__ float sum_range(const float *v, int64_t e0, int64_t e1, int gl) {
    constexpr int LH = __builtin_ctz(HP);
    constexpr int K = kTileK;
    const int64_t n = (e1 - e0) << LH;
    const float *vr = v + (e0 << LH);
    float part = 0.0f;
    for (int64_t t0 = 0; t0 < n; t0 += G * K) {
        float x[K];
        load_tile<G, K>(vr, n, t0, gl, 0.0f, x);
#pragma unroll
        for (int k = 0; k < K; ++k) part += x[k];
    }
    return part;
}

template <int G, int HP>
__global__ __launch_bounds__(kBlock) void k_row_sum(EdgeParams p, const float *v, float eps,
                                                    int accum, float *out, int32_t thr) {
    GALA_ROW_PROLOGUE(G);
    const bool mine = row_ok && !hub_row(p, thr, row);
    float part = 0.0f;
    if (mine) {
        for (int s = 0; s < p.seg.n; ++s) {
            int64_t e0, e1;
            row_range(p, s, row, e0, e1);
            part += sum_range<G, HP>(v, e0, e1, gl);
        }
    }
    part = head_sum<G, HP>(part);
    if (mine && gl < HP) {
        // reference: each segment's sum starts at 1e-12 (cuda.h:512,666)
        float r = part + (float)p.seg.n * eps;
        if (accum) r = out[row * HP + gl] + r;
        out[row * HP + gl] = r;
    }
}

// hub rows: per-chunk head sums of v -> ws[c][h]
template <int G, int HP>
__global__ __launch_bounds__(kBlock) void k_row_sum_chunk(EdgeParams p, const float *v, HubSplit sp) {
    GALA_CHUNK_PROLOGUE(G);
    const float part = head_sum<G, HP>(sum_range<G, HP>(v, e0, e1, gl));
    if (gl < HP) sp.ws[c * sp.ws_cols + gl] = part;
}

// hub rows: out[row, h] (+)= eps + the chunk sums in chunk order
__global__ __launch_bounds__(kBlock) void k_row_sum_fixup(EdgeParams p, float eps, int accum,
                                                          float *out, HubSplit sp) {
    const int H = p.heads;
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= sp.n_rows_split * H) return;
    const int64_t ri = t / H;
    const int h = (int)(t % H);
    float r = 0.0f;
    for (int64_t cc = sp.row_chunk0[ri]; cc < sp.row_chunk0[ri + 1]; ++cc) r += sp.ws[cc * sp.ws_cols + h];
    r = r + eps;
    const int64_t o = (int64_t)sp.rows[ri] * H + h;
    if (accum) r = out[o] + r;
    out[o] = r;
}

template <int G, int HP>
__device__ __forceinline__ void scale_range(float *v, float qv, int64_t e0, int64_t e1, int gl) {
    constexpr int LH = __builtin_ctz(HP);
    constexpr int K = kTileK;
    const int64_t n = (e1 - e0) << LH;
    float *vr = v + (e0 << LH);
    for (int64_t t0 = 0; t0 < n; t0 += G * K) {
        float x[K];
        load_tile<G, K>(vr, n, t0, gl, 0.0f, x);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int64_t t = t0 + gl + (int64_t)k * G;
            if (t < n) vr[t] = __fmul_rn(x[k], qv);
        }
    }
}

template <int G, int HP>
__global__ __launch_bounds__(kBlock) void k_row_scale(EdgeParams p, const float *q, float *v, int32_t thr) {
    GALA_ROW_PROLOGUE(G);
    if (!row_ok || hub_row(p, thr, row)) return;
    const float qv = q[row * HP + (gl & (HP - 1))];
    for (int s = 0; s < p.seg.n; ++s) {
        int64_t e0, e1;
        row_range(p, s, row, e0, e1);
        scale_range<G, HP>(v, qv, e0, e1, gl);
    }
}

template <int G, int HP>
__global__ __launch_bounds__(kBlock) void k_row_scale_chunk(EdgeParams p, const float *q, float *v,
                                                            HubSplit sp) {
    GALA_CHUNK_PROLOGUE(G);
    scale_range<G, HP>(v, q[row * HP + (gl & (HP - 1))], e0, e1, gl);
}

__device__ __forceinline__ float ref_exp(float s) {
    // torch::exp then torch::clamp(0, 1e12) (common.h:760-761); NaN propagates like clamp
    const float p = expf(s);
    return p > 1e12f ? 1e12f : p;
}

// softmax statistics of the logits [e0*HP, e1*HP): REF sum of clamped exp terms, FIXED an
// online (max, sum); x keeps the last tile
template <int G, int HP, int MODE>
__device__ __forceinline__ void softmax_stats(const float *logit, int64_t e0, int64_t e1, int gl,
                                              float &m, float &sum, float (&x)[kTileK]) {
    constexpr int LH = __builtin_ctz(HP);
    constexpr int K = kTileK;
    const int64_t n = (e1 - e0) << LH;
    const float *lr = logit + (e0 << LH);
    for (int64_t t0 = 0; t0 < n; t0 += G * K) {
        load_tile<G, K>(lr, n, t0, gl, -INFINITY, x);  // exp(-inf) = 0: fill is inert
        if (MODE == GALA_SOFTMAX_REF) {
#pragma unroll
            for (int k = 0; k < K; ++k) sum += ref_exp(x[k]);
        } else {
            float mt = x[0];
#pragma unroll
            for (int k = 1; k < K; ++k) mt = fmaxf(mt, x[k]);
            if (mt > m) {  // online max / sum
                sum = (m == -INFINITY) ? 0.0f : sum * expf(m - mt);
                m = mt;
            }
            if (m != -INFINITY) {
#pragma unroll
                for (int k = 0; k < K; ++k) sum += expf(x[k] - m);
            }
        }
    }
}

// the lanes' (m, sum) -> the head's (m, sum) (all lanes of the head get it)
template <int G, int HP, int MODE>
__device__ __forceinline__ void softmax_reduce(float &m, float &sum) {
    if (MODE == GALA_SOFTMAX_REF) {
        sum = head_sum<G, HP>(sum);
    } else {
        const float gm = head_max<G, HP>(m);
        sum = (m == -INFINITY) ? 0.0f : sum * expf(m - gm);
        sum = head_sum<G, HP>(sum);
        m = gm;
    }
}

template <int G, int HP, int MODE>
__device__ __forceinline__ void softmax_write(const float *logit, float *alpha, int64_t e0, int64_t e1,
                                              int gl, float m, float q) {
    constexpr int LH = __builtin_ctz(HP);
    constexpr int K = kTileK;
    const int64_t n = (e1 - e0) << LH;
    const float *lr = logit + (e0 << LH);
    float *ar = alpha + (e0 << LH);
    for (int64_t t0 = 0; t0 < n; t0 += G * K) {
        float x[K];
        load_tile<G, K>(lr, n, t0, gl, -INFINITY, x);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int64_t t = t0 + gl + (int64_t)k * G;
            const float pe = (MODE == GALA_SOFTMAX_REF) ? ref_exp(x[k]) : expf(x[k] - m);
            if (t < n) ar[t] = __fmul_rn(pe, q);
        }
    }
}

template <int G, int HP, int MODE>
__global__ __launch_bounds__(kBlock) void k_softmax_fwd(EdgeParams p, const float *logit,
                                                        float *alpha, int32_t thr) {
    GALA_ROW_PROLOGUE(G);
    constexpr int LH = __builtin_ctz(HP);
    constexpr int K = kTileK;
    const bool mine = row_ok && !hub_row(p, thr, row);
    float m = -INFINITY, sum = 0.0f;
    float x[K];
    bool in_regs = false;  // the whole row is in x[] (one segment, one tile)
    if (mine) {
        for (int s = 0; s < p.seg.n; ++s) {
            int64_t e0, e1;
            row_range(p, s, row, e0, e1);
            in_regs = p.seg.n == 1 && ((e1 - e0) << LH) <= G * K;
            softmax_stats<G, HP, MODE>(logit, e0, e1, gl, m, sum, x);
        }
    }
    softmax_reduce<G, HP, MODE>(m, sum);
    const float q = (MODE == GALA_SOFTMAX_REF) ? 1.0f / (sum + (float)p.seg.n * 1e-12f)  // torch::reciprocal
                                               : 1.0f / sum;
    if (!mine) return;
    if (in_regs) {
        int64_t e0, e1;
        row_range(p, 0, row, e0, e1);
        const int64_t n = (e1 - e0) << LH;
        float *ar = alpha + (e0 << LH);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int64_t t = gl + (int64_t)k * G;
            const float pe = (MODE == GALA_SOFTMAX_REF) ? ref_exp(x[k]) : expf(x[k] - m);
            if (t < n) ar[t] = __fmul_rn(pe, q);
        }
        return;
    }
    for (int s = 0; s < p.seg.n; ++s) {
        int64_t e0, e1;
        row_range(p, s, row, e0, e1);
        softmax_write<G, HP, MODE>(logit, alpha, e0, e1, gl, m, q);
    }
}

// hub rows: per-chunk head (m, sum) -> ws[c] = {m[HP], sum[HP]}
template <int G, int HP, int MODE>
__global__ __launch_bounds__(kBlock) void k_softmax_fwd_chunk(EdgeParams p, const float *logit, HubSplit sp) {
    GALA_CHUNK_PROLOGUE(G);
    float m = -INFINITY, sum = 0.0f, x[kTileK];
    softmax_stats<G, HP, MODE>(logit, e0, e1, gl, m, sum, x);
    softmax_reduce<G, HP, MODE>(m, sum);
    if (gl < HP) {
        sp.ws[c * sp.ws_cols + gl] = m;
        sp.ws[c * sp.ws_cols + HP + gl] = sum;
    }
}

// hub rows: merge the chunks' (m, sum) in chunk order -> the row's (m, q) in ws[c0]
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_softmax_fwd_fixup(EdgeParams p, HubSplit sp) {
    const int H = p.heads;
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= sp.n_rows_split * H) return;
    const int64_t ri = t / H;
    const int h = (int)(t % H);
    const int64_t c0 = sp.row_chunk0[ri];
    float m = -INFINITY, sum = 0.0f;
    for (int64_t cc = c0; cc < sp.row_chunk0[ri + 1]; ++cc) {
        const float mc = sp.ws[cc * sp.ws_cols + h], sc = sp.ws[cc * sp.ws_cols + H + h];
        if (MODE == GALA_SOFTMAX_REF) {
            sum += sc;
        } else if (mc != -INFINITY) {
            const float mn = fmaxf(m, mc);
            sum = ((m == -INFINITY) ? 0.0f : sum * expf(m - mn)) + sc * expf(mc - mn);
            m = mn;
        }
    }
    const float q = (MODE == GALA_SOFTMAX_REF) ? 1.0f / (sum + 1e-12f) : 1.0f / sum;
    sp.ws[c0 * sp.ws_cols + h] = m;
    sp.ws[c0 * sp.ws_cols + H + h] = q;
}

// hub rows: alpha of one chunk with its row's (m, q)
template <int G, int HP, int MODE>
__global__ __launch_bounds__(kBlock) void k_softmax_fwd_chunk2(EdgeParams p, const float *logit, float *alpha,
                                                               HubSplit sp) {
    GALA_CHUNK_PROLOGUE(G);
    const int h = gl & (HP - 1);
    const float *w0 = sp.ws + (int64_t)sp.row_chunk0[ri] * sp.ws_cols;
    softmax_write<G, HP, MODE>(logit, alpha, e0, e1, gl, w0[h], w0[HP + h]);
}

template <int G, int HP>
__device__ __forceinline__ float dot_range(const float *a, const float *b, int64_t e0, int64_t e1, int gl,
                                           float (&av)[kTileK], float (&dv)[kTileK]) {
    constexpr int LH = __builtin_ctz(HP);
    constexpr int K = kTileK;
    const int64_t n = (e1 - e0) << LH;
    const int64_t o = e0 << LH;
    float part = 0.0f;
    for (int64_t t0 = 0; t0 < n; t0 += G * K) {
        load_tile<G, K>(a + o, n, t0, gl, 0.0f, av);
        load_tile<G, K>(b + o, n, t0, gl, 0.0f, dv);
#pragma unroll
        for (int k = 0; k < K; ++k) part += __fmul_rn(av[k], dv[k]);
    }
    return part;
}

template <int G, int HP>
__device__ __forceinline__ void softmax_bwd_write(const float *alpha, const float *dalpha, float *dlogit,
                                                  int64_t e0, int64_t e1, int gl, float acc,
                                                  float (&a)[kTileK], float (&d)[kTileK], bool in_regs) {
    constexpr int LH = __builtin_ctz(HP);
    constexpr int K = kTileK;
    const int64_t n = (e1 - e0) << LH;
    const int64_t o = e0 << LH;
    for (int64_t t0 = 0; t0 < n; t0 += G * K) {
        if (!in_regs) {
            load_tile<G, K>(alpha + o, n, t0, gl, 0.0f, a);
            load_tile<G, K>(dalpha + o, n, t0, gl, 0.0f, d);
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int64_t t = t0 + gl + (int64_t)k * G;
            const float sds = __fmul_rn(a[k], d[k]);
            if (t < n) dlogit[o + t] = __fsub_rn(sds, __fmul_rn(a[k], acc));  // sds - K8(acc)
        }
    }
}

template <int G, int HP, int MODE>
__global__ __launch_bounds__(kBlock) void k_softmax_bwd(EdgeParams p, const float *alpha,
                                                        const float *dalpha, float *dlogit, int32_t thr) {
    GALA_ROW_PROLOGUE(G);
    constexpr int LH = __builtin_ctz(HP);
    constexpr int K = kTileK;
    const bool mine = row_ok && !hub_row(p, thr, row);
    const float eps = (MODE == GALA_SOFTMAX_REF) ? 1e-12f : 0.0f;
    float part = 0.0f;
    float a[K], d[K];
    bool in_regs = false;
    if (mine) {
        for (int s = 0; s < p.seg.n; ++s) {
            int64_t e0, e1;
            row_range(p, s, row, e0, e1);
            in_regs = p.seg.n == 1 && ((e1 - e0) << LH) <= G * K;
            part += dot_range<G, HP>(alpha, dalpha, e0, e1, gl, a, d);
        }
    }
    part = head_sum<G, HP>(part);
    const float acc = part + (float)p.seg.n * eps;  // K7 on sds (common.h:793-794)
    if (!mine) return;
    for (int s = 0; s < p.seg.n; ++s) {
        int64_t e0, e1;
        row_range(p, s, row, e0, e1);
        softmax_bwd_write<G, HP>(alpha, dalpha, dlogit, e0, e1, gl, acc, a, d, in_regs);
    }
}

// hub rows: per-chunk head sums of alpha * d_alpha -> ws[c][h]
template <int G, int HP>
__global__ __launch_bounds__(kBlock) void k_softmax_bwd_chunk(EdgeParams p, const float *alpha,
                                                              const float *dalpha, HubSplit sp) {
    GALA_CHUNK_PROLOGUE(G);
    float a[kTileK], d[kTileK];
    const float part = head_sum<G, HP>(dot_range<G, HP>(alpha, dalpha, e0, e1, gl, a, d));
    if (gl < HP) sp.ws[c * sp.ws_cols + gl] = part;
}

// hub rows: acc = eps + the chunk sums in chunk order -> ws[c0][HP + h]
__global__ __launch_bounds__(kBlock) void k_softmax_bwd_fixup(EdgeParams p, float eps, HubSplit sp) {
    const int H = p.heads;
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= sp.n_rows_split * H) return;
    const int64_t ri = t / H;
    const int h = (int)(t % H);
    const int64_t c0 = sp.row_chunk0[ri];
    float r = 0.0f;
    for (int64_t cc = c0; cc < sp.row_chunk0[ri + 1]; ++cc) r += sp.ws[cc * sp.ws_cols + h];
    sp.ws[c0 * sp.ws_cols + H + h] = r + eps;
}

template <int G, int HP>
__global__ __launch_bounds__(kBlock) void k_softmax_bwd_chunk2(EdgeParams p, const float *alpha,
                                                               const float *dalpha, float *dlogit,
                                                               HubSplit sp) {
    GALA_CHUNK_PROLOGUE(G);
    const float acc = sp.ws[(int64_t)sp.row_chunk0[ri] * sp.ws_cols + HP + (gl & (HP - 1))];
    float a[kTileK], d[kTileK];
    softmax_bwd_write<G, HP>(alpha, dalpha, dlogit, e0, e1, gl, acc, a, d, false);
}

// ---- generic-heads variants (runtime head count, per-head passes) ---------------------
// ---- SDDVV --------------------------------------------------------------------------
template <int G, int OP>
__global__ __launch_bounds__(kBlock) void k_sddvv_generic(EdgeParams p, const float *a, const float *b,
                                                  float slope, float *out) {
    GALA_ROW_PROLOGUE(G);
    if (!row_ok) return;
    const int H = p.heads;
    for (int s = 0; s < p.seg.n; ++s) {
        int64_t e0, e1;
        row_range(p, s, row, e0, e1);
        const int64_t n = (e1 - e0) * H;
        for (int64_t t = gl; t < n; t += G) {
            const int64_t e = e0 + t / H;
            const int h = (int)(t % H);
            const float av = a[row * H + h];
            const float bv = b[(int64_t)p.col[e] * H + h];
            float r;
            if (OP == GALA_SDDVV_MUL) {
                r = __fmul_rn(av, bv);
            } else {
                r = __fadd_rn(av, bv);
                if (OP == GALA_SDDVV_ADD_LRELU) r = r > 0.0f ? r : __fmul_rn(r, slope);
            }
            out[e * H + h] = r;
        }
    }
}

// ---- edge -> row sum (K7) ----------------------------------------------------------
template <int G>
__global__ __launch_bounds__(kBlock) void k_row_sum_generic(EdgeParams p, const float *v, float eps,
                                                    int accum, float *out) {
    GALA_ROW_PROLOGUE(G);
    const int H = p.heads;
    for (int h = 0; h < H; ++h) {
        float part = 0.0f;
        if (row_ok) {
            for (int s = 0; s < p.seg.n; ++s) {
                int64_t e0, e1;
                row_range(p, s, row, e0, e1);
                for (int64_t e = e0 + gl; e < e1; e += G) part += v[e * H + h];
            }
        }
        part = group_sum<G>(part);
        if (row_ok && gl == 0) {
            // reference: each segment's sum starts at 1e-12 (cuda.h:512,666)
            float r = part + (float)p.seg.n * eps;
            if (accum) r = out[row * H + h] + r;
            out[row * H + h] = r;
        }
    }
}

// ---- row -> edge scale (K8) --------------------------------------------------------
template <int G>
__global__ __launch_bounds__(kBlock) void k_row_scale_generic(EdgeParams p, const float *q, float *v) {
    GALA_ROW_PROLOGUE(G);
    if (!row_ok) return;
    const int H = p.heads;
    for (int s = 0; s < p.seg.n; ++s) {
        int64_t e0, e1;
        row_range(p, s, row, e0, e1);
        const int64_t n = (e1 - e0) * H;
        for (int64_t t = gl; t < n; t += G) {
            const int64_t idx = e0 * H + t;
            v[idx] = __fmul_rn(v[idx], q[row * H + (int)(t % H)]);
        }
    }
}

// ---- edge softmax -------------------------------------------------------------------

template <int G, int MODE>
__global__ __launch_bounds__(kBlock) void k_softmax_fwd_generic(EdgeParams p, const float *logit,
                                                        float *alpha) {
    GALA_ROW_PROLOGUE(G);
    const int H = p.heads;
    for (int h = 0; h < H; ++h) {
        float m = -INFINITY, sum = 0.0f;
        if (row_ok) {
            for (int s = 0; s < p.seg.n; ++s) {
                int64_t e0, e1;
                row_range(p, s, row, e0, e1);
                for (int64_t e = e0 + gl; e < e1; e += G) {
                    const float x = logit[e * H + h];
                    if (MODE == GALA_SOFTMAX_REF) {
                        sum += ref_exp(x);
                    } else {  // online max/sum
                        if (x > m) {
                            sum = sum * expf(m - x) + 1.0f;
                            m = x;
                        } else {
                            sum += expf(x - m);
                        }
                    }
                }
            }
        }
        float q;
        if (MODE == GALA_SOFTMAX_REF) {
            sum = group_sum<G>(sum);
            q = 1.0f / (sum + (float)p.seg.n * 1e-12f);  // torch::reciprocal(row_sum)
        } else {
            const float gm = group_max<G>(m);
            sum = (m == -INFINITY) ? 0.0f : sum * expf(m - gm);
            sum = group_sum<G>(sum);
            m = gm;
            q = 1.0f / sum;
        }
        if (!row_ok) continue;
        for (int s = 0; s < p.seg.n; ++s) {
            int64_t e0, e1;
            row_range(p, s, row, e0, e1);
            for (int64_t e = e0 + gl; e < e1; e += G) {
                const float x = logit[e * H + h];
                const float pe = (MODE == GALA_SOFTMAX_REF) ? ref_exp(x) : expf(x - m);
                alpha[e * H + h] = __fmul_rn(pe, q);
            }
        }
    }
}

template <int G, int MODE>
__global__ __launch_bounds__(kBlock) void k_softmax_bwd_generic(EdgeParams p, const float *alpha,
                                                        const float *dalpha, float *dlogit) {
    GALA_ROW_PROLOGUE(G);
    const int H = p.heads;
    const float eps = (MODE == GALA_SOFTMAX_REF) ? 1e-12f : 0.0f;
    for (int h = 0; h < H; ++h) {
        float part = 0.0f;
        if (row_ok) {
            for (int s = 0; s < p.seg.n; ++s) {
                int64_t e0, e1;
                row_range(p, s, row, e0, e1);
                for (int64_t e = e0 + gl; e < e1; e += G)
                    part += __fmul_rn(alpha[e * H + h], dalpha[e * H + h]);
            }
        }
        part = group_sum<G>(part);
        const float acc = part + (float)p.seg.n * eps;  // K7 on sds (common.h:793-794)
        if (!row_ok) continue;
        for (int s = 0; s < p.seg.n; ++s) {
            int64_t e0, e1;
            row_range(p, s, row, e0, e1);
            for (int64_t e = e0 + gl; e < e1; e += G) {
                const float a = alpha[e * H + h];
                const float sds = __fmul_rn(a, dalpha[e * H + h]);
                dlogit[e * H + h] = __fsub_rn(sds, __fmul_rn(a, acc));  // sds - K8(acc)
            }
        }
    }
}

// ---- SDDMM dot (K9) -----------------------------------------------------------------
// Row group of G lanes over the features (VEC per lane); U edges per batch have all
// their loads in flight before the dot products.  For one head (HW == G) the U partial
// dots are reduced with a reduce-scatter butterfly (U-1 + log2(G/U) shuffles per batch,
// lane k*(G/U) ends with edge k); with heads each head reduces over its HW lanes.
template <int G, int U>
__device__ __forceinline__ float reduce_scatter(float (&v)[U], int gl) {
#pragma unroll
    for (int m = U, o = G / 2; m > 1; m >>= 1, o >>= 1) {
        const bool up = (gl & o) != 0;
#pragma unroll
        for (int i = 0; i < m / 2; ++i) {
            const float send = up ? v[i] : v[i + m / 2];
            const float keep = up ? v[i + m / 2] : v[i];
            v[i] = keep + __shfl_xor(send, o, 64);
        }
    }
    float r = v[0];
#pragma unroll
    for (int o = G / (2 * U); o >= 1; o >>= 1) r += __shfl_xor(r, o, 64);
    return r;
}

// Feature ownership of one lane inside a row group: CH chunks of VEC floats at
// (ch*G + gl)*VEC.  CH > 1 is used for one head whose row is not a multiple of 4 floats
// (F = 47, the Products class count: VEC = 1), so that 16 lanes, not 64, share a row.
template <int G, int VEC, int CH>
struct Lanes {
    bool valid[CH];
    int64_t off[CH];
    int nv[CH];  // real columns of the lane's vector: VEC, fewer in a padded row's last one
    __device__ __forceinline__ Lanes(int gl, int32_t F) {
#pragma unroll
        for (int ch = 0; ch < CH; ++ch) {
            const int f = (ch * G + gl) * VEC;
            valid[ch] = f < F;
            off[ch] = valid[ch] ? f : 0;  // lanes past F read a valid column, never store
            nv[ch] = valid[ch] ? (F - f < VEC ? F - f : VEC) : 0;
        }
    }
    // element i of vector ch is a real column (padding columns are read but zeroed before
    // any dot product, and never written)
    __device__ __forceinline__ bool in(int ch, int i) const { return i < nv[ch]; }
};

// fp32 vectors of VEC lanes' worth of features
template <int VEC>
struct GVec;
template <>
struct GVec<1> { typedef float T; };
template <>
struct GVec<2> { typedef float T __attribute__((ext_vector_type(2))); };
template <>
struct GVec<4> { typedef float T __attribute__((ext_vector_type(4))); };

// A gathered vector with its padding columns (element i >= nv) zeroed: padding may hold
// anything, and 0 * Inf would reach a dot product.
template <int VEC, typename V>
__device__ __forceinline__ V mask_pad(int nv, V v) {
    if (nv < VEC) {
        float *e = reinterpret_cast<float *>(&v);
#pragma unroll
        for (int i = 0; i < VEC; ++i) e[i] = i < nv ? e[i] : 0.0f;
    }
    return v;
}

// Edges [e0, e1) of `row` (one row group): out[e] = <Ad[row], Bd[col_e]> per head.
template <int G, int VEC, int HW, int U, int CH = 1>
__device__ __forceinline__ void sddmm_range(const EdgeParams &p, int gl, bool row_ok, int64_t row,
                                            const float *Ad, int64_t lda, const float *Bd,
                                            int64_t ldb, int32_t F, float *out, int64_t e0,
                                            int64_t e1) {
    const Lanes<G, VEC, CH> ln(gl, F);
    const bool cv = row_ok && ln.valid[0];
    float a[CH][VEC];
#pragma unroll
    for (int ch = 0; ch < CH; ++ch)
#pragma unroll
        for (int i = 0; i < VEC; ++i) a[ch][i] = (row_ok && ln.in(ch, i)) ? Ad[row * lda + ln.off[ch] + i] : 0.0f;
    const int H = p.heads;
    const int D = F / H;
    const int h = cv ? (int)(ln.off[0] / D) : 0;
    const int32_t n = (int32_t)(e1 - e0);
    for (int32_t j0 = 0; j0 < n; j0 += U) {
        float part[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int32_t j = (j0 + k < n) ? j0 + k : n - 1;
            const int64_t c = p.col[e0 + j];
            const float *bp = Bd + c * ldb;
            float acc = 0.0f;
#pragma unroll
            for (int ch = 0; ch < CH; ++ch) {
                typedef typename GVec<VEC>::T V;
                const V bv = mask_pad<VEC>(ln.nv[ch], *reinterpret_cast<const V *>(bp + ln.off[ch]));
#pragma unroll
                for (int i = 0; i < VEC; ++i) acc = fmaf(a[ch][i], reinterpret_cast<const float *>(&bv)[i], acc);
            }
            part[k] = acc;
        }
        if (HW == G) {
            const float r = reduce_scatter<G, U>(part, gl);
            const int k = gl / (G / U);
            if ((gl & (G / U - 1)) == 0 && j0 + k < n) out[e0 + j0 + k] = r;
        } else {
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const float r = group_sum<HW>(part[k]);
                if (cv && (gl % HW) == 0 && j0 + k < n) out[(e0 + j0 + k) * H + h] = r;
            }
        }
    }
}

// hub rows (A->split): one row group per chunk of a split row; no fix-up needed
template <int G, int VEC, int HW, int U, int CH>
__global__ __launch_bounds__(kBlock) void k_sddmm_chunk(EdgeParams p, const float *Ad, int64_t lda,
                                                        const float *Bd, int64_t ldb, int32_t F,
                                                        float *out, const int32_t *rows,
                                                        const int32_t *row_chunk0,
                                                        const int32_t *chunk_row, int64_t n_chunks,
                                                        int32_t chunk) {
    const int lane = threadIdx.x & (kWave - 1);
    const int gl = lane & (G - 1);
    const int64_t c = ((int64_t)blockIdx.x * (kBlock / kWave) + threadIdx.x / kWave) * (kWave / G) + lane / G;
    if (c >= n_chunks) return;  // whole groups exit together
    const int32_t ri = chunk_row[c];
    const int64_t row = rows[ri];
    const int64_t r0 = p.rowptr[row], r1 = p.rowptr[row + 1];
    const int64_t e0 = r0 + (c - row_chunk0[ri]) * (int64_t)chunk;
    const int64_t e1 = (e0 + chunk < r1) ? e0 + chunk : r1;
    sddmm_range<G, VEC, HW, U, CH>(p, gl, true, row, Ad, lda, Bd, ldb, F, out, e0, e1);
}

template <int G, int VEC, int HW, int U, int CH>
__global__ __launch_bounds__(kBlock) void k_sddmm(EdgeParams p, const float *Ad, int64_t lda,
                                                  const float *Bd, int64_t ldb, int32_t F,
                                                  float *out, int32_t split_threshold) {
    GALA_ROW_PROLOGUE(G);
    if (split_threshold > 0) {
        // rows of one group share the row: the skip is uniform inside every group
        if (row_ok && p.rowptr[row + 1] - p.rowptr[row] > split_threshold) return;
    }
    for (int s = 0; s < p.seg.n; ++s) {
        int64_t e0 = 0, e1 = 0;
        if (row_ok) row_range(p, s, row, e0, e1);
        sddmm_range<G, VEC, HW, U, CH>(p, gl, row_ok, row, Ad, lda, Bd, ldb, F, out, e0, e1);
    }
}

// ---- fused GAT aggregation -----------------------------------------------------------
// Row group of G lanes, lane g owns CH x VEC features (Lanes); U edges per batch: cols,
// aR[col] and the X row slices are all loaded before the softmax updates.

// RC (one head): the source logit aR[col] = <X[col,:], wR> + bR is recomputed from the X
// row the aggregation gathers anyway (the DSL's attnR = dsl.nn.ffn(res, out=1) of the
// aggregated `res`, tests/GALA-DSL/gat/*), instead of a separate random aR[col] read.
template <int G, int VEC, int CH>
__device__ __forceinline__ float attn_dot(const float (&w)[CH][VEC],
                                          const typename GVec<VEC>::T (&x)[CH]) {
    float d = 0.0f;
#pragma unroll
    for (int ch = 0; ch < CH; ++ch) {
        const float *xv = reinterpret_cast<const float *>(&x[ch]);
#pragma unroll
        for (int i = 0; i < VEC; ++i) d = fmaf(w[ch][i], xv[i], d);
    }
    return group_sum<G>(d);
}

template <int G, int VEC, int CH>
__device__ __forceinline__ void load_attn(const Lanes<G, VEC, CH> &ln, const float *wR,
                                          float (&w)[CH][VEC]) {
#pragma unroll
    for (int ch = 0; ch < CH; ++ch)
#pragma unroll
        for (int i = 0; i < VEC; ++i) w[ch][i] = ln.in(ch, i) ? wR[ln.off[ch] + i] : 0.0f;
}

// Operands of the fused GAT kernels (forward and backward).
struct GatDev {
    const float *aL, *aR, *wR, *bR;  // aR == nullptr: recompute aR from X, wR, bR (RC)
    const float *X;
    const float *dY, *alpha;         // backward
    float *Y, *alpha_out;            // forward
    float *d_logit, *d_aL;           // backward
    int64_t ldx, ldy, lddy;
    int32_t F;
    float slope;
};


// The lane's share of one row (or one chunk of a hub row) for the GAT kernels.
template <int G, int VEC, int CH, bool RC>
struct GatLane {
    Lanes<G, VEC, CH> ln;
    int H, D, hh;
    bool cv, leader;
    float al, wb;
    float w[CH][VEC];
    __device__ __forceinline__ GatLane(const EdgeParams &p, const GatDev &d, int gl, int64_t row)
        : ln(gl, d.F) {
        H = p.heads;  // CH > 1 and RC only with H == 1
        D = d.F / H;
        cv = ln.valid[0];
        hh = (int)(ln.off[0] / D);
        leader = cv && (ln.off[0] % D) == 0;
        al = d.aL[row * H + hh];
        wb = 0.0f;
        if (RC) {
            load_attn<G, VEC, CH>(ln, d.wR, w);
            wb = d.bR ? d.bR[0] : 0.0f;
        }
    }
};

// Running state of the forward for one row / chunk: per lane CH x VEC accumulators and the
// head's (max, sum) of the softmax (FIXED: online, relative to m; REF: plain sums).
template <int VEC, int CH>
struct FwdState {
    float acc[CH][VEC];
    float m, sum;
    __device__ __forceinline__ FwdState() : m(-INFINITY), sum(0.0f) {
#pragma unroll
        for (int ch = 0; ch < CH; ++ch)
#pragma unroll
            for (int i = 0; i < VEC; ++i) acc[ch][i] = 0.0f;
    }
};

// Edges [e0, e1) of `row` into the forward state.  When `park`, the head leader lane parks
// each edge's exp term (REF) or logit (FIXED) in alpha_out for the alpha pass.
template <int G, int VEC, int U, int MODE, int CH, bool RC>
__device__ __forceinline__ void gat_fwd_range(const EdgeParams &p, const GatDev &d,
                                              const GatLane<G, VEC, CH, RC> &gl_, bool park,
                                              int64_t e0, int64_t e1, FwdState<VEC, CH> &st) {
    typedef typename GVec<VEC>::T V;
    const int H = gl_.H, hh = gl_.hh;
    const bool leader = park && gl_.leader;
    const int32_t n = (int32_t)(e1 - e0);
    for (int32_t j0 = 0; j0 < n; j0 += U) {
        int64_t c[U];
        float ar[U];
        V x[U][CH];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int32_t j = (j0 + k < n) ? j0 + k : n - 1;
            c[k] = p.col[e0 + j];
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            if (!RC) ar[k] = d.aR[c[k] * H + hh];
#pragma unroll
            for (int ch = 0; ch < CH; ++ch)
                x[k][ch] = mask_pad<VEC>(gl_.ln.nv[ch], *reinterpret_cast<const V *>(d.X + c[k] * d.ldx + gl_.ln.off[ch]));
        }
        if (RC) {
#pragma unroll
            for (int k = 0; k < U; ++k) ar[k] = __fadd_rn(attn_dot<G, VEC, CH>(gl_.w, x[k]), gl_.wb);
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            if (j0 + k >= n) continue;
            float z = __fadd_rn(gl_.al, ar[k]);
            z = z > 0.0f ? z : __fmul_rn(z, d.slope);
            if (MODE == GALA_SOFTMAX_REF) {
                const float pe = ref_exp(z);
                if (leader) d.alpha_out[(e0 + j0 + k) * H + hh] = pe;
                st.sum = __fadd_rn(st.sum, pe);
#pragma unroll
                for (int ch = 0; ch < CH; ++ch) {
                    const float *xv = reinterpret_cast<const float *>(&x[k][ch]);
#pragma unroll
                    for (int i = 0; i < VEC; ++i) st.acc[ch][i] = fmaf(pe, xv[i], st.acc[ch][i]);
                }
                continue;
            }
            if (leader) d.alpha_out[(e0 + j0 + k) * H + hh] = z;
            if (z > st.m) {
                const float r = expf(st.m - z);
                st.sum = fmaf(st.sum, r, 1.0f);
#pragma unroll
                for (int ch = 0; ch < CH; ++ch) {
                    const float *xv = reinterpret_cast<const float *>(&x[k][ch]);
#pragma unroll
                    for (int i = 0; i < VEC; ++i) st.acc[ch][i] = fmaf(st.acc[ch][i], r, xv[i]);
                }
                st.m = z;
            } else {
                const float pe = expf(z - st.m);
                st.sum = __fadd_rn(st.sum, pe);
#pragma unroll
                for (int ch = 0; ch < CH; ++ch) {
                    const float *xv = reinterpret_cast<const float *>(&x[k][ch]);
#pragma unroll
                    for (int i = 0; i < VEC; ++i) st.acc[ch][i] = fmaf(pe, xv[i], st.acc[ch][i]);
                }
            }
        }
    }
}

// Y[row] = acc * q with q = 1 / (sum [+ S * 1e-12 in REF mode]); returns q.
template <int G, int VEC, int CH, bool RC, int MODE>
__device__ __forceinline__ float gat_fwd_store(const GatDev &d, const GatLane<G, VEC, CH, RC> &gl_,
                                               int64_t row, int nseg, const FwdState<VEC, CH> &st) {
    typedef typename GVec<VEC>::T V;
    const float den = (MODE == GALA_SOFTMAX_REF) ? st.sum + (float)nseg * 1e-12f : st.sum;
    const float q = 1.0f / den;
#pragma unroll
    for (int ch = 0; ch < CH; ++ch) {
        if (!gl_.ln.valid[ch]) continue;
        V out;
        float *ov = reinterpret_cast<float *>(&out);
#pragma unroll
        for (int i = 0; i < VEC; ++i)
            ov[i] = (MODE != GALA_SOFTMAX_REF && st.sum == 0.0f) ? 0.0f : __fmul_rn(st.acc[ch][i], q);
        float *yp = d.Y + row * d.ldy + gl_.ln.off[ch];
        if (gl_.ln.nv[ch] == VEC) {
            *reinterpret_cast<V *>(yp) = out;
        } else {  // a padded row's last vector: its real columns only
#pragma unroll
            for (int i = 0; i < VEC; ++i)
                if (gl_.ln.in(ch, i)) yp[i] = ov[i];
        }
    }
    return q;
}

// alpha of the parked (edge, head) values [t0, t1) of one row: lane g handles head g % H
// (H | G) with that head's (m, q)
template <int G, int MODE>
__device__ __forceinline__ void gat_alpha_rescale(float *ar, int64_t n, int gl, float mh, float qh) {
    constexpr int K = kTileK;
    for (int64_t t0 = 0; t0 < n; t0 += G * K) {
        float v[K];
        load_tile<G, K>(ar, n, t0, gl, 0.0f, v);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int64_t t = t0 + gl + (int64_t)k * G;
            const float pe = (MODE == GALA_SOFTMAX_REF) ? v[k] : expf(v[k] - mh);
            if (t < n) ar[t] = __fmul_rn(pe, qh);
        }
    }
}

// One pass per row: logits, LeakyReLU, softmax (REF exp-clamp / FIXED online max), the
// alpha-weighted aggregation, then 1/sum; alpha (if requested) in a parked-value pass.
template <int G, int VEC, int U, int MODE, int CH, bool RC>
__global__ __launch_bounds__(kBlock) void k_gat_fwd(EdgeParams p, GatDev d, int32_t split_threshold) {
    GALA_ROW_PROLOGUE(G);
    if (!row_ok) return;
    if (split_threshold > 0 && p.rowptr[row + 1] - p.rowptr[row] > split_threshold)
        return;  // hub row: k_gat_fwd_chunk / _fixup / k_gat_alpha_chunk
    const GatLane<G, VEC, CH, RC> gl_(p, d, gl, row);
    const int H = gl_.H, D = gl_.D;
    // With H | G the main pass parks each (edge, head)'s exp term (REF) or logit (FIXED)
    // in alpha_out (the head's first lane writes it) and the alpha pass rescales it in
    // place: a contiguous re-read of the row instead of a second col -> aR gather.
    const bool park = d.alpha_out != nullptr && (G % H) == 0;
    FwdState<VEC, CH> st;
    for (int s = 0; s < p.seg.n; ++s) {
        int64_t e0, e1;
        row_range(p, s, row, e0, e1);
        gat_fwd_range<G, VEC, U, MODE, CH, RC>(p, d, gl_, park, e0, e1, st);
    }
    const float q = gat_fwd_store<G, VEC, CH, RC, MODE>(d, gl_, row, p.seg.n, st);
    if (!d.alpha_out) return;
    const int gbase = (threadIdx.x & (kWave - 1)) & ~(G - 1);
    if (park) {
        const int h = gl % H;
        const int src = gbase + (h * D) / VEC;
        const float mh = __shfl(st.m, src, 64);
        const float qh = __shfl(q, src, 64);
        // the parked values were stored by other lanes of this wave
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        for (int s = 0; s < p.seg.n; ++s) {
            int64_t e0, e1;
            row_range(p, s, row, e0, e1);
            gat_alpha_rescale<G, MODE>(d.alpha_out + e0 * H, (e1 - e0) * H, gl, mh, qh);
        }
        return;
    }
    // heads that do not divide G: per head, lanes stride the row's edges (aR re-read)
    for (int s = 0; s < p.seg.n; ++s) {
        int64_t e0, e1;
        row_range(p, s, row, e0, e1);
        for (int hd = 0; hd < H; ++hd) {
            const int src = gbase + (hd * D) / VEC;
            const float mh = __shfl(st.m, src, 64);
            const float qh = __shfl(q, src, 64);
            const float alh = d.aL[row * H + hd];
            for (int64_t e = e0 + gl; e < e1; e += G) {
                float z = __fadd_rn(alh, d.aR[(int64_t)p.col[e] * H + hd]);
                z = z > 0.0f ? z : __fmul_rn(z, d.slope);
                const float pe = (MODE == GALA_SOFTMAX_REF) ? ref_exp(z) : expf(z - mh);
                d.alpha_out[e * H + hd] = __fmul_rn(pe, qh);
            }
        }
    }
}


// hub rows, forward: chunk partial state -> ws[c] = {acc[F], m[H], sum[H]}
template <int G, int VEC, int U, int MODE, int CH, bool RC>
__global__ __launch_bounds__(kBlock) void k_gat_fwd_chunk(EdgeParams p, GatDev d, HubSplit sp) {
    GALA_CHUNK_PROLOGUE(G);
    const GatLane<G, VEC, CH, RC> gl_(p, d, gl, row);
    FwdState<VEC, CH> st;
    gat_fwd_range<G, VEC, U, MODE, CH, RC>(p, d, gl_, d.alpha_out != nullptr, e0, e1, st);
    float *w = sp.ws + c * sp.ws_cols;
#pragma unroll
    for (int ch = 0; ch < CH; ++ch)
#pragma unroll
        for (int i = 0; i < VEC; ++i)
            if (gl_.ln.in(ch, i)) w[gl_.ln.off[ch] + i] = st.acc[ch][i];
    if (gl_.leader) {
        w[d.F + gl_.hh] = st.m;
        w[d.F + gl_.H + gl_.hh] = st.sum;
    }
}

// hub rows, forward: combine the chunk partials in chunk order, store Y; (m, q) of every
// head go to the row's first chunk slot for k_gat_alpha_chunk
template <int G, int VEC, int MODE, int CH, bool RC>
__global__ __launch_bounds__(kBlock) void k_gat_fwd_fixup(EdgeParams p, GatDev d, HubSplit sp) {
    const int lane = threadIdx.x & (kWave - 1);
    const int gl = lane & (G - 1);
    const int64_t ri = ((int64_t)blockIdx.x * (kBlock / kWave) + threadIdx.x / kWave) * (kWave / G) + lane / G;
    if (ri >= sp.n_rows_split) return;
    const int64_t row = sp.rows[ri];
    const GatLane<G, VEC, CH, RC> gl_(p, d, gl, row);
    const int F = d.F, H = gl_.H, hh = gl_.hh;
    FwdState<VEC, CH> st;
    const int64_t c0 = sp.row_chunk0[ri], c1 = sp.row_chunk0[ri + 1];
    for (int64_t cc = c0; cc < c1; ++cc) {
        const float *w = sp.ws + cc * sp.ws_cols;
        const float mc = w[F + hh], sc = w[F + H + hh];
        float a = 1.0f, b = 1.0f;
        if (MODE != GALA_SOFTMAX_REF) {
            if (mc == -INFINITY) continue;  // no edges in this chunk's partial
            const float mn = fmaxf(st.m, mc);
            a = (st.m == -INFINITY) ? 0.0f : expf(st.m - mn);
            b = expf(mc - mn);
            st.m = mn;
            st.sum = fmaf(st.sum, a, __fmul_rn(sc, b));
        } else {
            st.sum = __fadd_rn(st.sum, sc);
        }
#pragma unroll
        for (int ch = 0; ch < CH; ++ch)
#pragma unroll
            for (int i = 0; i < VEC; ++i) {
                const float v = gl_.ln.in(ch, i) ? w[gl_.ln.off[ch] + i] : 0.0f;
                st.acc[ch][i] = (MODE == GALA_SOFTMAX_REF) ? __fadd_rn(st.acc[ch][i], v)
                                                           : fmaf(st.acc[ch][i], a, __fmul_rn(v, b));
            }
    }
    const float q = gat_fwd_store<G, VEC, CH, RC, MODE>(d, gl_, row, 1, st);
    if (gl_.leader && d.alpha_out) {
        float *w0 = sp.ws + c0 * sp.ws_cols;
        w0[F + hh] = st.m;
        w0[F + H + hh] = q;
    }
}

// hub rows, forward: alpha of one chunk's parked values with its row's (m, q)
template <int G, int VEC, int MODE>
__global__ __launch_bounds__(kBlock) void k_gat_alpha_chunk(EdgeParams p, GatDev d, HubSplit sp) {
    GALA_CHUNK_PROLOGUE(G);
    const int H = p.heads;
    const int h = gl % H;
    const float *w0 = sp.ws + (int64_t)sp.row_chunk0[ri] * sp.ws_cols;
    gat_alpha_rescale<G, MODE>(d.alpha_out + e0 * H, (e1 - e0) * H, gl, w0[d.F + h], w0[d.F + H + h]);
}

// ---- fused GAT backward -------------------------------------------------------------
// Row group of G lanes over the features (Lanes: CH x VEC per lane), HW lanes per head.
// Pass 1: U edges per batch load col, X row slice, aR[col,h] and alpha before the
// head-wise dot reductions; every lane of a head then holds d_alpha and accumulates the
// head's sum(sds) (and, in REF mode, sum(m*sds) and sum(m*alpha)).  FIXED mode parks sds
// in d_logit (head leader lane) and a second, contiguous (edge, head) pass forms dz.
struct BwdState {
    float acc = 0.0f, s_msds = 0.0f, s_ma = 0.0f;
};

template <int G, int VEC, int U, int HW, int MODE, int CH, bool RC>
__device__ __forceinline__ void gat_bwd_range(const EdgeParams &p, const GatDev &d,
                                              const GatLane<G, VEC, CH, RC> &gl_,
                                              const float (&dy)[CH][VEC], int64_t e0, int64_t e1,
                                              BwdState &st) {
    typedef typename GVec<VEC>::T V;
    const int H = gl_.H, hh = gl_.hh;
    const int32_t n = (int32_t)(e1 - e0);
    for (int32_t j0 = 0; j0 < n; j0 += U) {
        int64_t c[U];
        float ar[U], a[U], part[U];
        V x[U][CH];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int32_t j = (j0 + k < n) ? j0 + k : n - 1;
            c[k] = p.col[e0 + j];
            a[k] = d.alpha[(e0 + j) * H + hh];
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            if (!RC) ar[k] = d.aR[c[k] * H + hh];
#pragma unroll
            for (int ch = 0; ch < CH; ++ch)
                x[k][ch] = mask_pad<VEC>(gl_.ln.nv[ch], *reinterpret_cast<const V *>(d.X + c[k] * d.ldx + gl_.ln.off[ch]));
        }
        if (RC) {
#pragma unroll
            for (int k = 0; k < U; ++k) ar[k] = __fadd_rn(attn_dot<G, VEC, CH>(gl_.w, x[k]), gl_.wb);
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            float dd = 0.0f;
#pragma unroll
            for (int ch = 0; ch < CH; ++ch) {
                const float *xv = reinterpret_cast<const float *>(&x[k][ch]);
#pragma unroll
                for (int i = 0; i < VEC; ++i) dd = fmaf(dy[ch][i], xv[i], dd);
            }
            part[k] = dd;
        }
#pragma unroll
        for (int k = 0; k < U; ++k) part[k] = group_sum<HW>(part[k]);
#pragma unroll
        for (int k = 0; k < U; ++k) {
            if (j0 + k >= n) continue;
            const float sds = __fmul_rn(a[k], part[k]);
            st.acc += sds;
            if (MODE == GALA_SOFTMAX_REF) {
                const bool pos = __fadd_rn(gl_.al, ar[k]) > 0.0f;
                st.s_msds += pos ? sds : __fmul_rn(sds, d.slope);
                st.s_ma += pos ? a[k] : __fmul_rn(a[k], d.slope);
            } else if (gl_.leader) {
                d.d_logit[(e0 + j0 + k) * H + hh] = sds;
            }
        }
    }
}

template <int G, int VEC, int CH, bool RC>
__device__ __forceinline__ void load_dy(const GatDev &d, const GatLane<G, VEC, CH, RC> &gl_, int64_t row,
                                        float (&dy)[CH][VEC]) {
    typedef typename GVec<VEC>::T V;
#pragma unroll
    for (int ch = 0; ch < CH; ++ch) {
        const V t = *reinterpret_cast<const V *>(d.dY + row * d.lddy + gl_.ln.off[ch]);
#pragma unroll
        for (int i = 0; i < VEC; ++i) dy[ch][i] = gl_.ln.in(ch, i) ? reinterpret_cast<const float *>(&t)[i] : 0.0f;
    }
}

// FIXED second pass over the parked sds of (edge, head) values [0, n) of one row slice:
// dz = LeakyReLU'(z) * (sds - alpha * acc_h); returns the lane's partial sum of dz
template <int G>
__device__ __forceinline__ float gat_bwd_dz(const EdgeParams &p, const GatDev &d, int64_t row,
                                            int64_t e0, int64_t n, int gl, int h, float acch) {
    constexpr int K = kTileK;
    const int H = p.heads;
    const float alh = d.aL[row * H + h];
    float *dl = d.d_logit + e0 * H;
    const float *ap = d.alpha + e0 * H;
    float rs = 0.0f;
    for (int64_t t0 = 0; t0 < n; t0 += G * K) {
        float sv[K], av[K], rv[K];
        int32_t cc[K];
        load_tile<G, K>(dl, n, t0, gl, 0.0f, sv);
        load_tile<G, K>(ap, n, t0, gl, 0.0f, av);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int64_t t = t0 + gl + (int64_t)k * G;
            cc[k] = p.col[e0 + (t < n ? t : 0) / H];
        }
#pragma unroll
        for (int k = 0; k < K; ++k) rv[k] = d.aR[(int64_t)cc[k] * H + h];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int64_t t = t0 + gl + (int64_t)k * G;
            if (t >= n) continue;
            const float ds = __fsub_rn(sv[k], __fmul_rn(av[k], acch));
            const float dz = __fadd_rn(alh, rv[k]) > 0.0f ? ds : __fmul_rn(ds, d.slope);
            dl[t] = dz;
            rs += dz;
        }
    }
    return rs;
}

template <int G, int VEC, int U, int HW, int MODE, int CH, bool RC>
__global__ __launch_bounds__(kBlock) void k_gat_bwd(EdgeParams p, GatDev d, int32_t split_threshold) {
    GALA_ROW_PROLOGUE(G);
    if (!row_ok) return;
    if (split_threshold > 0 && p.rowptr[row + 1] - p.rowptr[row] > split_threshold)
        return;  // hub row: k_gat_bwd_chunk / _fixup (/ _chunk2 / _fixup2)
    const GatLane<G, VEC, CH, RC> gl_(p, d, gl, row);
    const int H = gl_.H, D = gl_.D;
    float dy[CH][VEC];
    load_dy<G, VEC, CH, RC>(d, gl_, row, dy);
    const float eps = (MODE == GALA_SOFTMAX_REF) ? 1e-12f : 0.0f;
    BwdState st;
    for (int s = 0; s < p.seg.n; ++s) {
        int64_t e0, e1;
        row_range(p, s, row, e0, e1);
        gat_bwd_range<G, VEC, U, HW, MODE, CH, RC>(p, d, gl_, dy, e0, e1, st);
    }
    const float acc = st.acc + (float)p.seg.n * eps;  // K7 on sds (common.h:793-794)
    if (MODE == GALA_SOFTMAX_REF) {
        // sum_row m*(sds - alpha*acc), then K7's 1e-12 per segment (common.h:662-667)
        if (gl_.leader) d.d_aL[row * H + gl_.hh] = (st.s_msds - acc * st.s_ma) + (float)p.seg.n * eps;
        return;
    }
    // FIXED: dz per (edge, head) from the parked sds; lane g keeps head g % H (H | G)
    const int gbase = lane & ~(G - 1);
    const int h = gl % H;
    const float acch = __shfl(acc, gbase + (h * D) / VEC, 64);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // parked by other lanes
    float rs = 0.0f;
    for (int s = 0; s < p.seg.n; ++s) {
        int64_t e0, e1;
        row_range(p, s, row, e0, e1);
        rs += gat_bwd_dz<G>(p, d, row, e0, (e1 - e0) * H, gl, h, acch);
    }
    for (int o = G / 2; o >= H; o >>= 1) rs += __shfl_xor(rs, o, 64);  // lanes of head h
    if (gl < H) d.d_aL[row * H + gl] = rs;
}

// hub rows, backward pass 1: chunk partials -> ws[c] = {acc[H], s_msds[H], s_ma[H]}
// (REF) or {acc[H]} with sds parked in d_logit (FIXED)
template <int G, int VEC, int U, int HW, int MODE, int CH, bool RC>
__global__ __launch_bounds__(kBlock) void k_gat_bwd_chunk(EdgeParams p, GatDev d, HubSplit sp) {
    GALA_CHUNK_PROLOGUE(G);
    const GatLane<G, VEC, CH, RC> gl_(p, d, gl, row);
    float dy[CH][VEC];
    load_dy<G, VEC, CH, RC>(d, gl_, row, dy);
    BwdState st;
    gat_bwd_range<G, VEC, U, HW, MODE, CH, RC>(p, d, gl_, dy, e0, e1, st);
    if (!gl_.leader) return;
    float *w = sp.ws + c * sp.ws_cols;
    const int H = gl_.H, hh = gl_.hh;
    w[hh] = st.acc;
    if (MODE == GALA_SOFTMAX_REF) {
        w[H + hh] = st.s_msds;
        w[2 * H + hh] = st.s_ma;
    }
}

// hub rows, backward: sum the chunk partials in chunk order.  REF: d_aL.  FIXED: the row's
// acc per head -> ws[c0][H + h] for k_gat_bwd_chunk2.  One thread per (split row, head).
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_gat_bwd_fixup(EdgeParams p, GatDev d, HubSplit sp) {
    const int H = p.heads;
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= sp.n_rows_split * H) return;
    const int64_t ri = t / H;
    const int h = (int)(t % H);
    const int64_t row = sp.rows[ri];
    const int64_t c0 = sp.row_chunk0[ri], c1 = sp.row_chunk0[ri + 1];
    float acc = 0.0f, s1 = 0.0f, s2 = 0.0f;
    for (int64_t cc = c0; cc < c1; ++cc) {
        const float *w = sp.ws + cc * sp.ws_cols;
        acc = __fadd_rn(acc, w[h]);
        if (MODE == GALA_SOFTMAX_REF) {
            s1 = __fadd_rn(s1, w[H + h]);
            s2 = __fadd_rn(s2, w[2 * H + h]);
        }
    }
    if (MODE == GALA_SOFTMAX_REF) {
        acc = __fadd_rn(acc, 1e-12f);
        d.d_aL[row * H + h] = (s1 - acc * s2) + 1e-12f;
    } else {
        sp.ws[c0 * sp.ws_cols + H + h] = acc;
    }
}

// hub rows, FIXED backward pass 2: dz of one chunk; partial row sums -> ws[c][2H + h]
template <int G>
__global__ __launch_bounds__(kBlock) void k_gat_bwd_chunk2(EdgeParams p, GatDev d, HubSplit sp) {
    GALA_CHUNK_PROLOGUE(G);
    const int H = p.heads;
    const int h = gl % H;
    const float acch = sp.ws[(int64_t)sp.row_chunk0[ri] * sp.ws_cols + H + h];
    float rs = gat_bwd_dz<G>(p, d, row, e0, (e1 - e0) * H, gl, h, acch);
    for (int o = G / 2; o >= H; o >>= 1) rs += __shfl_xor(rs, o, 64);
    if (gl < H) sp.ws[c * sp.ws_cols + 2 * H + gl] = rs;
}

// hub rows, FIXED backward: d_aL = the chunks' dz sums in chunk order
__global__ __launch_bounds__(kBlock) void k_gat_bwd_fixup2(EdgeParams p, GatDev d, HubSplit sp) {
    const int H = p.heads;
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= sp.n_rows_split * H) return;
    const int64_t ri = t / H;
    const int h = (int)(t % H);
    float rs = 0.0f;
    for (int64_t cc = sp.row_chunk0[ri]; cc < sp.row_chunk0[ri + 1]; ++cc)
        rs = __fadd_rn(rs, sp.ws[cc * sp.ws_cols + 2 * H + h]);
    d.d_aL[(int64_t)sp.rows[ri] * H + h] = rs;
}

__global__ __launch_bounds__(kBlock) void k_permute(const int32_t *perm, const float *src,
                                                    int64_t n, int32_t H, float *dst) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= n * H) return;
    const int64_t i = t / H;
    const int h = (int)(t % H);
    dst[t] = src[(int64_t)perm[i] * H + h];
}

// ---- host side ------------------------------------------------------------------------
static int pick_group(const gala_csr_t *A, int heads) {
    // lanes per row from the mean row length (edges*heads)
    // ~2-4 edges per lane: several rows per wave amortise the per-row bookkeeping
    const double avg = A->n_rows ? (double)A->nnz * heads / (double)A->n_rows : 1.0;
    int g = 4;
    while (g < 64 && 2 * g * 2 <= avg) g <<= 1;
    return g;
}

// lanes per row for the register-tiled kernels: the smallest group whose tile (G*K
// values) holds a mean row with 15 % slack, so most rows take one tile
static int pick_group_tiled(const gala_csr_t *A, int heads) {
    const double avg = A->n_rows ? (double)A->nnz * heads / (double)A->n_rows : 1.0;
    int g = 4;
    while (g < 64 && (double)g * kTileK < 1.15 * avg) g <<= 1;
    return g;
}

// One head whose row is not a multiple of 4 floats (VEC < 4) and spans 17..64 vectors:
// 16 lanes own ceil(L/16) chunks each (Lanes), instead of 64 lanes one vector each, so 4
// rows share a wave and the per-edge softmax / reduction work is not repeated 64-fold.
// Returns the chunk count (1 = the one-vector-per-lane layout).
// F rounded up to a multiple of v (a padded row's width)
static int64_t pad_to(int64_t F, int v) { return (F + v - 1) / v * v; }

static int narrow_chunks(int heads, int vec, int L) {
    return (heads == 1 && vec < 4 && L > 16 && L <= 64) ? (L + 15) / 16 : 1;
}

static int edge_setup(const gala_csr_t *A, int32_t heads, EdgeParams *p) {
    int st = check_csr(A);
    if (st) return st;
    if (heads < 1) return GALA_ERR_INVALID_ARG;
    if (A->n_seg > kMaxSegPerLaunch) return GALA_ERR_UNSUPPORTED;
    p->rowptr = A->rowptr;
    p->col = A->col;
    p->n_rows = A->n_rows;
    p->heads = heads;
    // XCD-aware row-block order (gala_internal.h); graphs with a hub / row-order plan are
    // skewed (heavy rows cluster in id order) and keep the hardware order.  Banded
    // Products-shaped graph, F = 32: SDDMM 1.83 -> 1.69 ms, GAT forward 1.65 -> 1.60 ms;
    // uniform: within 1 % either way
    p->xcd_order = A->split == nullptr;
    return fill_segments(A, 0, &p->seg);
}

static unsigned blocks_for(int64_t n_rows, int G) {
    const int64_t rpb = (int64_t)(kBlock / kWave) * (kWave / G);
    return (unsigned)((n_rows + rpb - 1) / rpb);
}

#define GALA_DISPATCH_G(G, ...)                        \
    switch (G) {                                       \
        case 4: { constexpr int GG = 4; __VA_ARGS__; } break;   \
        case 8: { constexpr int GG = 8; __VA_ARGS__; } break;   \
        case 16: { constexpr int GG = 16; __VA_ARGS__; } break; \
        case 32: { constexpr int GG = 32; __VA_ARGS__; } break; \
        default: { constexpr int GG = 64; __VA_ARGS__; } break; \
    }

// heads as a compile-time power of two (0 = not supported by the flattened kernels)
static int pow2_heads(int heads) {
    return (heads == 1 || heads == 2 || heads == 4 || heads == 8 || heads == 16) ? heads : 0;
}

#define GALA_CASE_HP(GV, ...)                                                              \
    switch (hp) {                                                                          \
        case 1: { constexpr int GG = GV, HH = 1; __VA_ARGS__; } break;                     \
        case 2: { constexpr int GG = GV, HH = (2 <= GV ? 2 : GV); __VA_ARGS__; } break;    \
        case 4: { constexpr int GG = GV, HH = (4 <= GV ? 4 : GV); __VA_ARGS__; } break;    \
        case 8: { constexpr int GG = GV, HH = (8 <= GV ? 8 : GV); __VA_ARGS__; } break;    \
        default: { constexpr int GG = GV, HH = (16 <= GV ? 16 : GV); __VA_ARGS__; } break; \
    }
#define GALA_DISPATCH_GH(G, ...)                           \
    switch (G) {                                           \
        case 4: GALA_CASE_HP(4, __VA_ARGS__) break;        \
        case 8: GALA_CASE_HP(8, __VA_ARGS__) break;        \
        case 16: GALA_CASE_HP(16, __VA_ARGS__) break;      \
        case 32: GALA_CASE_HP(32, __VA_ARGS__) break;      \
        default: GALA_CASE_HP(64, __VA_ARGS__) break;      \
    }

}  // namespace gala

using namespace gala;

static unsigned blocks_for_groups(int64_t n, int G) {
    const int64_t per_block = (int64_t)(kBlock / kWave) * (kWave / G);
    return (unsigned)((n + per_block - 1) / per_block);
}

// the hub-row plan of A, when it applies and its workspace holds `need` floats per chunk
// (otherwise hub rows run in one pass, like every other row)
static bool hub_split(const gala_csr_t *A, int64_t need, HubSplit *sp) {
    const gala_split_plan_t *plan = A->split;
    if (!plan || plan->n_chunks <= 0 || A->n_seg != 1 || !plan->rows || !plan->row_chunk0 ||
        !plan->chunk_row || (need > 0 && (!plan->workspace || plan->ws_cols < need)) || plan->chunk < 1 ||
        plan->threshold < 1)
        return false;
    sp->rows = plan->rows;
    sp->row_chunk0 = plan->row_chunk0;
    sp->chunk_row = plan->chunk_row;
    sp->ws = plan->workspace;
    sp->ws_cols = plan->ws_cols;
    sp->n_chunks = plan->n_chunks;
    sp->n_rows_split = plan->n_rows_split;
    sp->chunk = plan->chunk;
    sp->threshold = plan->threshold;
    return true;
}

extern "C" int gala_sddvv_f32(const gala_csr_t *A, const float *a_row, const float *b_col,
                              int32_t heads, int32_t op, float slope, float *out_e,
                              void *stream) {
    EdgeParams p;
    int st = edge_setup(A, heads, &p);
    if (st) return st;
    if (op < GALA_SDDVV_ADD || op > GALA_SDDVV_ADD_LRELU) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0 || A->nnz == 0) return GALA_OK;
    if (!a_row || !b_col || !out_e) return GALA_ERR_INVALID_ARG;
    hipStream_t hs = (hipStream_t)stream;
    const int hp = pow2_heads(heads);
    if (hp) {
        const int G = std::max(pick_group_tiled(A, heads), hp);
        const dim3 grid(blocks_for(A->n_rows, G));
        HubSplit sp{};
        const bool split = hub_split(A, 0, &sp);
        const int32_t thr = split ? sp.threshold : 0;
#define GALA_SDDVV_OP(OPV)                                                                          \
    {                                                                                                \
        hipLaunchKernelGGL((k_sddvv<GG, HH, OPV>), grid, dim3(kBlock), 0, hs, p, a_row, b_col, slope, out_e, thr); \
        if (split)                                                                                   \
            hipLaunchKernelGGL((k_sddvv_chunk<GG, HH, OPV>), dim3(blocks_for_groups(sp.n_chunks, GG)), dim3(kBlock), \
                               0, hs, p, a_row, b_col, slope, out_e, sp);                            \
    }
        GALA_DISPATCH_GH(G, {
            if (op == GALA_SDDVV_ADD) GALA_SDDVV_OP(GALA_SDDVV_ADD)
            else if (op == GALA_SDDVV_MUL) GALA_SDDVV_OP(GALA_SDDVV_MUL)
            else GALA_SDDVV_OP(GALA_SDDVV_ADD_LRELU)
        });
#undef GALA_SDDVV_OP
        return launch_status();
    }
    const int G = pick_group(A, heads);
    GALA_DISPATCH_G(G, {
        const dim3 grid(blocks_for(A->n_rows, GG));
        if (op == GALA_SDDVV_ADD)
            hipLaunchKernelGGL((k_sddvv_generic<GG, GALA_SDDVV_ADD>), grid, dim3(kBlock), 0, hs, p, a_row, b_col, slope, out_e);
        else if (op == GALA_SDDVV_MUL)
            hipLaunchKernelGGL((k_sddvv_generic<GG, GALA_SDDVV_MUL>), grid, dim3(kBlock), 0, hs, p, a_row, b_col, slope, out_e);
        else
            hipLaunchKernelGGL((k_sddvv_generic<GG, GALA_SDDVV_ADD_LRELU>), grid, dim3(kBlock), 0, hs, p, a_row, b_col, slope, out_e);
    });
    return launch_status();
}

extern "C" int gala_row_sum_f32(const gala_csr_t *A, const float *v_e, int32_t heads, float eps,
                                float *out_row, int32_t flags, void *stream) {
    EdgeParams p;
    int st = edge_setup(A, heads, &p);
    if (st) return st;
    if (flags & ~GALA_SPMM_ACCUM) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0) return GALA_OK;
    if (!out_row || (!v_e && A->nnz > 0)) return GALA_ERR_INVALID_ARG;
    const int accum = (flags & GALA_SPMM_ACCUM) ? 1 : 0;
    hipStream_t hs = (hipStream_t)stream;
    const int hp = pow2_heads(heads);
    if (hp) {
        const int G = std::max(pick_group_tiled(A, heads), hp);
        const dim3 grid(blocks_for(A->n_rows, G));
        HubSplit sp{};
        const bool split = hub_split(A, 2 * (int64_t)hp, &sp);
        const int32_t thr = split ? sp.threshold : 0;
        GALA_DISPATCH_GH(G, {
            hipLaunchKernelGGL((k_row_sum<GG, HH>), grid, dim3(kBlock), 0, hs, p, v_e, eps, accum, out_row, thr);
            if (split) {
                hipLaunchKernelGGL((k_row_sum_chunk<GG, HH>), dim3(blocks_for_groups(sp.n_chunks, GG)), dim3(kBlock),
                                   0, hs, p, v_e, sp);
                hipLaunchKernelGGL(k_row_sum_fixup, dim3((unsigned)((sp.n_rows_split * hp + kBlock - 1) / kBlock)),
                                   dim3(kBlock), 0, hs, p, eps, accum, out_row, sp);
            }
        });
        return launch_status();
    }
    const int G = pick_group(A, 1);
    GALA_DISPATCH_G(G, hipLaunchKernelGGL((k_row_sum_generic<GG>), dim3(blocks_for(A->n_rows, GG)),
                                          dim3(kBlock), 0, hs, p, v_e, eps, accum, out_row));
    return launch_status();
}

extern "C" int gala_row_scale_f32(const gala_csr_t *A, const float *q_row, int32_t heads,
                                  float *v_inout, void *stream) {
    EdgeParams p;
    int st = edge_setup(A, heads, &p);
    if (st) return st;
    if (A->n_rows == 0 || A->nnz == 0) return GALA_OK;
    if (!q_row || !v_inout) return GALA_ERR_INVALID_ARG;
    hipStream_t hs = (hipStream_t)stream;
    const int hp = pow2_heads(heads);
    if (hp) {
        const int G = std::max(pick_group_tiled(A, heads), hp);
        const dim3 grid(blocks_for(A->n_rows, G));
        HubSplit sp{};
        const bool split = hub_split(A, 0, &sp);
        const int32_t thr = split ? sp.threshold : 0;
        GALA_DISPATCH_GH(G, {
            hipLaunchKernelGGL((k_row_scale<GG, HH>), grid, dim3(kBlock), 0, hs, p, q_row, v_inout, thr);
            if (split)
                hipLaunchKernelGGL((k_row_scale_chunk<GG, HH>), dim3(blocks_for_groups(sp.n_chunks, GG)), dim3(kBlock),
                                   0, hs, p, q_row, v_inout, sp);
        });
        return launch_status();
    }
    const int G = pick_group(A, heads);
    GALA_DISPATCH_G(G, hipLaunchKernelGGL((k_row_scale_generic<GG>), dim3(blocks_for(A->n_rows, GG)),
                                          dim3(kBlock), 0, hs, p, q_row, v_inout));
    return launch_status();
}

extern "C" int gala_edge_softmax_fwd_f32(const gala_csr_t *A, const float *logits,
                                         int32_t heads, int32_t mode, float *alpha,
                                         void *stream) {
    EdgeParams p;
    int st = edge_setup(A, heads, &p);
    if (st) return st;
    if (mode != GALA_SOFTMAX_REF && mode != GALA_SOFTMAX_FIXED) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0 || A->nnz == 0) return GALA_OK;
    if (!logits || !alpha) return GALA_ERR_INVALID_ARG;
    hipStream_t hs = (hipStream_t)stream;
    const int hp = pow2_heads(heads);
    if (hp) {
        const int G = std::max(pick_group_tiled(A, heads), hp);
        const dim3 grid(blocks_for(A->n_rows, G));
        HubSplit sp{};
        const bool split = hub_split(A, 2 * (int64_t)hp, &sp);
        const int32_t thr = split ? sp.threshold : 0;
        const unsigned cb = split ? blocks_for_groups(sp.n_chunks, G) : 0;
        const unsigned tb = split ? (unsigned)((sp.n_rows_split * hp + kBlock - 1) / kBlock) : 0;
#define GALA_SMF(MODEV)                                                                              \
    {                                                                                                \
        hipLaunchKernelGGL((k_softmax_fwd<GG, HH, MODEV>), grid, dim3(kBlock), 0, hs, p, logits, alpha, thr); \
        if (split) {                                                                                 \
            hipLaunchKernelGGL((k_softmax_fwd_chunk<GG, HH, MODEV>), dim3(cb), dim3(kBlock), 0, hs, p, logits, sp); \
            hipLaunchKernelGGL((k_softmax_fwd_fixup<MODEV>), dim3(tb), dim3(kBlock), 0, hs, p, sp);  \
            hipLaunchKernelGGL((k_softmax_fwd_chunk2<GG, HH, MODEV>), dim3(cb), dim3(kBlock), 0, hs, p, logits, \
                               alpha, sp);                                                           \
        }                                                                                            \
    }
        GALA_DISPATCH_GH(G, {
            if (mode == GALA_SOFTMAX_REF) GALA_SMF(GALA_SOFTMAX_REF)
            else GALA_SMF(GALA_SOFTMAX_FIXED)
        });
#undef GALA_SMF
        return launch_status();
    }
    const int G = pick_group(A, 1);
    GALA_DISPATCH_G(G, {
        const dim3 grid(blocks_for(A->n_rows, GG));
        if (mode == GALA_SOFTMAX_REF)
            hipLaunchKernelGGL((k_softmax_fwd_generic<GG, GALA_SOFTMAX_REF>), grid, dim3(kBlock), 0, hs, p, logits, alpha);
        else
            hipLaunchKernelGGL((k_softmax_fwd_generic<GG, GALA_SOFTMAX_FIXED>), grid, dim3(kBlock), 0, hs, p, logits, alpha);
    });
    return launch_status();
}

extern "C" int gala_edge_softmax_bwd_f32(const gala_csr_t *A, const float *alpha,
                                         const float *d_alpha, int32_t heads, int32_t mode,
                                         float *d_logits, void *stream) {
    EdgeParams p;
    int st = edge_setup(A, heads, &p);
    if (st) return st;
    if (mode != GALA_SOFTMAX_REF && mode != GALA_SOFTMAX_FIXED) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0 || A->nnz == 0) return GALA_OK;
    if (!alpha || !d_alpha || !d_logits) return GALA_ERR_INVALID_ARG;
    hipStream_t hs = (hipStream_t)stream;
    const int hp = pow2_heads(heads);
    if (hp) {
        const int G = std::max(pick_group_tiled(A, heads), hp);
        const dim3 grid(blocks_for(A->n_rows, G));
        HubSplit sp{};
        const bool split = hub_split(A, 2 * (int64_t)hp, &sp);
        const int32_t thr = split ? sp.threshold : 0;
        const unsigned cb = split ? blocks_for_groups(sp.n_chunks, G) : 0;
        const unsigned tb = split ? (unsigned)((sp.n_rows_split * hp + kBlock - 1) / kBlock) : 0;
        const float eps = (mode == GALA_SOFTMAX_REF) ? 1e-12f : 0.0f;
        GALA_DISPATCH_GH(G, {
            if (mode == GALA_SOFTMAX_REF)
                hipLaunchKernelGGL((k_softmax_bwd<GG, HH, GALA_SOFTMAX_REF>), grid, dim3(kBlock), 0, hs, p, alpha, d_alpha, d_logits, thr);
            else
                hipLaunchKernelGGL((k_softmax_bwd<GG, HH, GALA_SOFTMAX_FIXED>), grid, dim3(kBlock), 0, hs, p, alpha, d_alpha, d_logits, thr);
            if (split) {
                hipLaunchKernelGGL((k_softmax_bwd_chunk<GG, HH>), dim3(cb), dim3(kBlock), 0, hs, p, alpha, d_alpha, sp);
                hipLaunchKernelGGL(k_softmax_bwd_fixup, dim3(tb), dim3(kBlock), 0, hs, p, eps, sp);
                hipLaunchKernelGGL((k_softmax_bwd_chunk2<GG, HH>), dim3(cb), dim3(kBlock), 0, hs, p, alpha, d_alpha,
                                   d_logits, sp);
            }
        });
        return launch_status();
    }
    const int G = pick_group(A, 1);
    GALA_DISPATCH_G(G, {
        const dim3 grid(blocks_for(A->n_rows, GG));
        if (mode == GALA_SOFTMAX_REF)
            hipLaunchKernelGGL((k_softmax_bwd_generic<GG, GALA_SOFTMAX_REF>), grid, dim3(kBlock), 0, hs, p, alpha, d_alpha, d_logits);
        else
            hipLaunchKernelGGL((k_softmax_bwd_generic<GG, GALA_SOFTMAX_FIXED>), grid, dim3(kBlock), 0, hs, p, alpha, d_alpha, d_logits);
    });
    return launch_status();
}

struct SddmmSplit {
    const int32_t *rows = nullptr, *row_chunk0 = nullptr, *chunk_row = nullptr;
    int64_t n_chunks = 0;
    int32_t chunk = 0, threshold = 0;
};

template <int G, int VEC, int HWV, int CH = 1>
static void launch_sddmm_hw(const EdgeParams &p, const SddmmSplit &sp, const float *Ad, int64_t lda,
                            const float *Bd, int64_t ldb, int32_t F, float *out, hipStream_t hs) {
    constexpr int U = (G >= 8) ? 8 : G;  // U <= G for the reduce-scatter
    constexpr int HW = (HWV < G) ? HWV : G;
    hipLaunchKernelGGL((k_sddmm<G, VEC, HW, U, CH>), dim3(blocks_for(p.n_rows, G)), dim3(kBlock), 0, hs,
                       p, Ad, lda, Bd, ldb, F, out, sp.threshold);
    if (sp.n_chunks > 0) {
        const int64_t per_block = (kBlock / kWave) * (kWave / G);
        hipLaunchKernelGGL((k_sddmm_chunk<G, VEC, HW, U, CH>), dim3((unsigned)((sp.n_chunks + per_block - 1) / per_block)),
                           dim3(kBlock), 0, hs, p, Ad, lda, Bd, ldb, F, out, sp.rows, sp.row_chunk0,
                           sp.chunk_row, sp.n_chunks, sp.chunk);
    }
}

template <int G, int VEC>
static void launch_sddmm(const EdgeParams &p, const SddmmSplit &sp, int hw, const float *Ad,
                         int64_t lda, const float *Bd, int64_t ldb, int32_t F, float *out,
                         hipStream_t hs) {
    switch (hw) {
        case 1: launch_sddmm_hw<G, VEC, 1>(p, sp, Ad, lda, Bd, ldb, F, out, hs); break;
        case 2: launch_sddmm_hw<G, VEC, 2>(p, sp, Ad, lda, Bd, ldb, F, out, hs); break;
        case 4: launch_sddmm_hw<G, VEC, 4>(p, sp, Ad, lda, Bd, ldb, F, out, hs); break;
        case 8: launch_sddmm_hw<G, VEC, 8>(p, sp, Ad, lda, Bd, ldb, F, out, hs); break;
        case 16: launch_sddmm_hw<G, VEC, 16>(p, sp, Ad, lda, Bd, ldb, F, out, hs); break;
        case 32: launch_sddmm_hw<G, VEC, 32>(p, sp, Ad, lda, Bd, ldb, F, out, hs); break;
        default: launch_sddmm_hw<G, VEC, G>(p, sp, Ad, lda, Bd, ldb, F, out, hs); break;
    }
}

template <int VEC>
static int sddmm_vec(const EdgeParams &p, const SddmmSplit &sp, int L, int hw, const float *Ad, int64_t lda,
                     const float *Bd, int64_t ldb, int32_t F, float *out, hipStream_t hs) {
    if (L <= 1) launch_sddmm<1, VEC>(p, sp, hw, Ad, lda, Bd, ldb, F, out, hs);
    else if (L <= 2) launch_sddmm<2, VEC>(p, sp, hw, Ad, lda, Bd, ldb, F, out, hs);
    else if (L <= 4) launch_sddmm<4, VEC>(p, sp, hw, Ad, lda, Bd, ldb, F, out, hs);
    else if (L <= 8) launch_sddmm<8, VEC>(p, sp, hw, Ad, lda, Bd, ldb, F, out, hs);
    else if (L <= 16) launch_sddmm<16, VEC>(p, sp, hw, Ad, lda, Bd, ldb, F, out, hs);
    else if (L <= 32) launch_sddmm<32, VEC>(p, sp, hw, Ad, lda, Bd, ldb, F, out, hs);
    else if (L <= 64) launch_sddmm<64, VEC>(p, sp, hw, Ad, lda, Bd, ldb, F, out, hs);
    else return GALA_ERR_UNSUPPORTED;
    return GALA_OK;
}

extern "C" int gala_sddmm_dot_f32(const gala_csr_t *A, const float *Ad, int64_t lda,
                                  const float *Bd, int64_t ldb, int32_t F, int32_t heads,
                                  float *out_e, void *stream) {
    EdgeParams p;
    int st = edge_setup(A, heads, &p);
    if (st) return st;
    if (F < 1 || F % heads != 0 || lda < F || ldb < F) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0 || A->nnz == 0) return GALA_OK;
    if (!Ad || !Bd || !out_e) return GALA_ERR_INVALID_ARG;
    const int D = F / heads;
    // VEC divides D (or, one head, fits padded rows: lda, ldb >= F rounded up to VEC), L =
    // lanes per row, the per-head lane count D/VEC must be a power of 2
    int vec = 4;
    while (vec > 1 && (!(D % vec == 0 || (heads == 1 && lda >= pad_to(F, vec) && ldb >= pad_to(F, vec))) ||
                       lda % vec || ldb % vec || ((uintptr_t)Ad % (4 * vec)) || ((uintptr_t)Bd % (4 * vec))))
        vec >>= 1;
    const int L = (F + vec - 1) / vec;
    const int hw_l = D / vec;
    int Gp = 1;
    while (Gp < L) Gp <<= 1;
    if (heads > 1 && (hw_l & (hw_l - 1))) return GALA_ERR_UNSUPPORTED;
    const int hw = heads > 1 ? hw_l : Gp;
    SddmmSplit sp;
    const gala_split_plan_t *plan = A->split;
    if (plan && plan->n_chunks > 0 && A->n_seg == 1) {
        if (!plan->rows || !plan->row_chunk0 || !plan->chunk_row || plan->chunk < 1)
            return GALA_ERR_INVALID_ARG;
        sp.rows = plan->rows;
        sp.row_chunk0 = plan->row_chunk0;
        sp.chunk_row = plan->chunk_row;
        sp.n_chunks = plan->n_chunks;
        sp.chunk = plan->chunk;
        sp.threshold = plan->threshold;
    }
    int r;
    const int ch = narrow_chunks(heads, vec, L);
    if (ch > 1) {
        hipStream_t hs = (hipStream_t)stream;
#define GALA_SD(V, C) launch_sddmm_hw<16, V, 16, C>(p, sp, Ad, lda, Bd, ldb, F, out_e, hs)
        if (vec == 2) {
            if (ch == 2) GALA_SD(2, 2); else if (ch == 3) GALA_SD(2, 3); else GALA_SD(2, 4);
        } else {
            if (ch == 2) GALA_SD(1, 2); else if (ch == 3) GALA_SD(1, 3); else GALA_SD(1, 4);
        }
#undef GALA_SD
        return launch_status();
    }
    if (vec == 4) r = sddmm_vec<4>(p, sp, L, hw, Ad, lda, Bd, ldb, F, out_e, (hipStream_t)stream);
    else if (vec == 2) r = sddmm_vec<2>(p, sp, L, hw, Ad, lda, Bd, ldb, F, out_e, (hipStream_t)stream);
    else r = sddmm_vec<1>(p, sp, L, hw, Ad, lda, Bd, ldb, F, out_e, (hipStream_t)stream);
    if (r) return r;
    return launch_status();
}

// Host-side launch description of the fused GAT kernels (forward and backward).
struct GatArgs {
    EdgeParams p;
    GatDev d;
    HubSplit sp;
    bool split;
    int mode;
    hipStream_t hs;
};


template <int G, int VEC, int CH, bool RC, int MODE>
static void launch_gat_mode(const GatArgs &a) {
    constexpr int U = 8;
    hipLaunchKernelGGL((k_gat_fwd<G, VEC, U, MODE, CH, RC>), dim3(blocks_for(a.p.n_rows, G)), dim3(kBlock),
                       0, a.hs, a.p, a.d, a.split ? a.sp.threshold : 0);
    if (!a.split) return;
    hipLaunchKernelGGL((k_gat_fwd_chunk<G, VEC, U, MODE, CH, RC>), dim3(blocks_for_groups(a.sp.n_chunks, G)),
                       dim3(kBlock), 0, a.hs, a.p, a.d, a.sp);
    hipLaunchKernelGGL((k_gat_fwd_fixup<G, VEC, MODE, CH, RC>), dim3(blocks_for_groups(a.sp.n_rows_split, G)),
                       dim3(kBlock), 0, a.hs, a.p, a.d, a.sp);
    if (a.d.alpha_out)
        hipLaunchKernelGGL((k_gat_alpha_chunk<G, VEC, MODE>), dim3(blocks_for_groups(a.sp.n_chunks, G)),
                           dim3(kBlock), 0, a.hs, a.p, a.d, a.sp);
}

template <int G, int VEC, int CH, bool RC>
static void launch_gat(const GatArgs &a) {
    if (a.mode == GALA_SOFTMAX_REF) launch_gat_mode<G, VEC, CH, RC, GALA_SOFTMAX_REF>(a);
    else launch_gat_mode<G, VEC, CH, RC, GALA_SOFTMAX_FIXED>(a);
}

template <int VEC, bool RC>
static int gat_vec(const GatArgs &a, int L, int ch) {
    if (ch == 2) launch_gat<16, VEC, 2, RC>(a);
    else if (ch == 3) launch_gat<16, VEC, 3, RC>(a);
    else if (ch == 4) launch_gat<16, VEC, 4, RC>(a);
    else if (L <= 1) launch_gat<1, VEC, 1, RC>(a);
    else if (L <= 2) launch_gat<2, VEC, 1, RC>(a);
    else if (L <= 4) launch_gat<4, VEC, 1, RC>(a);
    else if (L <= 8) launch_gat<8, VEC, 1, RC>(a);
    else if (L <= 16) launch_gat<16, VEC, 1, RC>(a);
    else if (L <= 32) launch_gat<32, VEC, 1, RC>(a);
    else if (L <= 64) launch_gat<64, VEC, 1, RC>(a);
    else return GALA_ERR_UNSUPPORTED;
    return GALA_OK;
}


static int gat_fwd_impl(const gala_csr_t *A, const float *aL, const float *aR, const float *wR,
                        const float *bR, const float *X, int64_t ldx, int32_t F, int32_t heads,
                        float slope, int32_t mode, float *Y, int64_t ldy, float *alpha_out,
                        void *stream) {
    GatArgs a{};
    int st = edge_setup(A, heads, &a.p);
    if (st) return st;
    if (mode != GALA_SOFTMAX_REF && mode != GALA_SOFTMAX_FIXED) return GALA_ERR_INVALID_ARG;
    if (F < 1 || F % heads != 0 || ldx < F || ldy < F) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0) return GALA_OK;
    if (!aL || (!aR && !wR) || !Y || (!X && A->nnz > 0)) return GALA_ERR_INVALID_ARG;
    const int D = F / heads;
    // VEC divides D, or (one head) fits padded rows: ldx, ldy >= F rounded up to VEC
    int vec = 4;
    while (vec > 1 && (!(D % vec == 0 || (heads == 1 && ldx >= pad_to(F, vec) && ldy >= pad_to(F, vec))) ||
                       ldx % vec || ldy % vec || ((uintptr_t)X % (4 * vec)) || ((uintptr_t)Y % (4 * vec))))
        vec >>= 1;
    const int L = (F + vec - 1) / vec;
    const int ch = narrow_chunks(heads, vec, L);
    int G = 16;
    if (ch == 1) {
        G = 1;
        while (G < L) G <<= 1;
    }
    a.mode = mode;
    a.d.aL = aL, a.d.aR = aR, a.d.wR = wR, a.d.bR = bR, a.d.X = X, a.d.ldx = ldx, a.d.F = F;
    a.d.slope = slope, a.d.Y = Y, a.d.ldy = ldy, a.d.alpha_out = alpha_out;
    a.hs = (hipStream_t)stream;
    a.split = (!alpha_out || G % heads == 0) && hub_split(A, (int64_t)F + 2 * heads, &a.sp);
    const bool rc = aR == nullptr;
    int r;
    if (vec == 4) r = rc ? gat_vec<4, true>(a, L, ch) : gat_vec<4, false>(a, L, ch);
    else if (vec == 2) r = rc ? gat_vec<2, true>(a, L, ch) : gat_vec<2, false>(a, L, ch);
    else r = rc ? gat_vec<1, true>(a, L, ch) : gat_vec<1, false>(a, L, ch);
    if (r) return r;
    return launch_status();
}

extern "C" int gala_gat_fwd_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                const float *X, int64_t ldx, int32_t F, int32_t heads,
                                float slope, int32_t mode, float *Y, int64_t ldy,
                                float *alpha_out, void *stream) {
    if (!aR && A && A->n_rows > 0) return GALA_ERR_INVALID_ARG;
    return gat_fwd_impl(A, aL, aR, nullptr, nullptr, X, ldx, F, heads, slope, mode, Y, ldy,
                        alpha_out, stream);
}

extern "C" int gala_gat_fwd_attn_f32(const gala_csr_t *A, const float *aL, const float *wR,
                                     const float *bR, const float *X, int64_t ldx, int32_t F,
                                     float slope, int32_t mode, float *Y, int64_t ldy,
                                     float *alpha_out, void *stream) {
    if (!wR && A && A->n_rows > 0) return GALA_ERR_INVALID_ARG;
    return gat_fwd_impl(A, aL, nullptr, wR, bR, X, ldx, F, 1, slope, mode, Y, ldy, alpha_out,
                        stream);
}

template <int G, int VEC, int HW, int CH, bool RC, int MODE>
static void launch_gat_bwd_mode(const GatArgs &a) {
    constexpr int U = 8;
    constexpr int HWc = (HW < G) ? HW : G;
    hipLaunchKernelGGL((k_gat_bwd<G, VEC, U, HWc, MODE, CH, RC>), dim3(blocks_for(a.p.n_rows, G)),
                       dim3(kBlock), 0, a.hs, a.p, a.d, a.split ? a.sp.threshold : 0);
    if (!a.split) return;
    const unsigned tb = (unsigned)((a.sp.n_rows_split * a.p.heads + kBlock - 1) / kBlock);
    hipLaunchKernelGGL((k_gat_bwd_chunk<G, VEC, U, HWc, MODE, CH, RC>), dim3(blocks_for_groups(a.sp.n_chunks, G)),
                       dim3(kBlock), 0, a.hs, a.p, a.d, a.sp);
    hipLaunchKernelGGL((k_gat_bwd_fixup<MODE>), dim3(tb), dim3(kBlock), 0, a.hs, a.p, a.d, a.sp);
    if (MODE == GALA_SOFTMAX_REF) return;
    hipLaunchKernelGGL((k_gat_bwd_chunk2<G>), dim3(blocks_for_groups(a.sp.n_chunks, G)), dim3(kBlock), 0,
                       a.hs, a.p, a.d, a.sp);
    hipLaunchKernelGGL(k_gat_bwd_fixup2, dim3(tb), dim3(kBlock), 0, a.hs, a.p, a.d, a.sp);
}

template <int G, int VEC, int HW, int CH, bool RC>
static void launch_gat_bwd(const GatArgs &a) {
    if (a.mode == GALA_SOFTMAX_REF) launch_gat_bwd_mode<G, VEC, HW, CH, RC, GALA_SOFTMAX_REF>(a);
    else if (!RC) launch_gat_bwd_mode<G, VEC, HW, CH, false, GALA_SOFTMAX_FIXED>(a);
    // FIXED + RC is refused by gat_bwd_impl: its second pass needs aR
}

template <int G, int VEC, bool RC>
static void gat_bwd_hw(const GatArgs &a, int hw) {
    switch (hw) {
        case 1: launch_gat_bwd<G, VEC, 1, 1, RC>(a); break;
        case 2: launch_gat_bwd<G, VEC, 2, 1, RC>(a); break;
        case 4: launch_gat_bwd<G, VEC, 4, 1, RC>(a); break;
        case 8: launch_gat_bwd<G, VEC, 8, 1, RC>(a); break;
        case 16: launch_gat_bwd<G, VEC, 16, 1, RC>(a); break;
        case 32: launch_gat_bwd<G, VEC, 32, 1, RC>(a); break;
        default: launch_gat_bwd<G, VEC, G, 1, RC>(a); break;
    }
}

template <int VEC, bool RC>
static int gat_bwd_vec(const GatArgs &a, int L, int hw, int ch) {
    if (ch == 2) launch_gat_bwd<16, VEC, 16, 2, RC>(a);
    else if (ch == 3) launch_gat_bwd<16, VEC, 16, 3, RC>(a);
    else if (ch == 4) launch_gat_bwd<16, VEC, 16, 4, RC>(a);
    else if (L <= 1) gat_bwd_hw<1, VEC, RC>(a, hw);
    else if (L <= 2) gat_bwd_hw<2, VEC, RC>(a, hw);
    else if (L <= 4) gat_bwd_hw<4, VEC, RC>(a, hw);
    else if (L <= 8) gat_bwd_hw<8, VEC, RC>(a, hw);
    else if (L <= 16) gat_bwd_hw<16, VEC, RC>(a, hw);
    else if (L <= 32) gat_bwd_hw<32, VEC, RC>(a, hw);
    else if (L <= 64) gat_bwd_hw<64, VEC, RC>(a, hw);
    else return GALA_ERR_UNSUPPORTED;
    return GALA_OK;
}

static int gat_bwd_impl(const gala_csr_t *A, const float *aL, const float *aR, const float *wR,
                        const float *bR, const float *X, int64_t ldx, const float *dY,
                        int64_t lddy, int32_t F, int32_t heads, float slope, int32_t mode,
                        const float *alpha, float *d_logit, float *d_aL, void *stream) {
    GatArgs a{};
    int st = edge_setup(A, heads, &a.p);
    if (st) return st;
    if (mode != GALA_SOFTMAX_REF && mode != GALA_SOFTMAX_FIXED) return GALA_ERR_INVALID_ARG;
    if (F < 1 || F % heads != 0 || ldx < F || lddy < F) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0) return GALA_OK;
    if (!aL || (!aR && !wR) || !dY || !d_aL || (A->nnz > 0 && (!X || !alpha)))
        return GALA_ERR_INVALID_ARG;
    if (mode == GALA_SOFTMAX_FIXED && !d_logit && A->nnz > 0) return GALA_ERR_INVALID_ARG;
    if (!aR && (mode != GALA_SOFTMAX_REF || heads != 1)) return GALA_ERR_UNSUPPORTED;
    const int D = F / heads;
    int vec = 4;
    while (vec > 1 && (!(D % vec == 0 || (heads == 1 && ldx >= pad_to(F, vec) && lddy >= pad_to(F, vec))) ||
                       ldx % vec || lddy % vec || ((uintptr_t)X % (4 * vec)) || ((uintptr_t)dY % (4 * vec))))
        vec >>= 1;
    const int L = (F + vec - 1) / vec;
    int G = 1;
    while (G < L) G <<= 1;
    const int hw_l = D / vec;
    if (heads > 1 && ((hw_l & (hw_l - 1)) || G % heads)) return GALA_ERR_UNSUPPORTED;
    if (mode == GALA_SOFTMAX_FIXED && G % heads) return GALA_ERR_UNSUPPORTED;
    const int hw = heads > 1 ? hw_l : G;
    const int ch = narrow_chunks(heads, vec, L);
    a.mode = mode;
    a.d.aL = aL, a.d.aR = aR, a.d.wR = wR, a.d.bR = bR, a.d.X = X, a.d.ldx = ldx, a.d.F = F;
    a.d.slope = slope, a.d.dY = dY, a.d.lddy = lddy, a.d.alpha = alpha, a.d.d_logit = d_logit;
    a.d.d_aL = d_aL;
    a.hs = (hipStream_t)stream;
    a.split = hub_split(A, 3 * (int64_t)heads, &a.sp);
    const bool rc = aR == nullptr;
    int r;
    if (vec == 4) r = rc ? gat_bwd_vec<4, true>(a, L, hw, ch) : gat_bwd_vec<4, false>(a, L, hw, ch);
    else if (vec == 2) r = rc ? gat_bwd_vec<2, true>(a, L, hw, ch) : gat_bwd_vec<2, false>(a, L, hw, ch);
    else r = rc ? gat_bwd_vec<1, true>(a, L, hw, ch) : gat_bwd_vec<1, false>(a, L, hw, ch);
    if (r) return r;
    return launch_status();
}

extern "C" int gala_gat_bwd_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                const float *X, int64_t ldx, const float *dY, int64_t lddy,
                                int32_t F, int32_t heads, float slope, int32_t mode,
                                const float *alpha, float *d_logit, float *d_aL, void *stream) {
    if (!aR && A && A->n_rows > 0) return GALA_ERR_INVALID_ARG;
    return gat_bwd_impl(A, aL, aR, nullptr, nullptr, X, ldx, dY, lddy, F, heads, slope, mode,
                        alpha, d_logit, d_aL, stream);
}

extern "C" int gala_gat_bwd_attn_f32(const gala_csr_t *A, const float *aL, const float *wR,
                                     const float *bR, const float *X, int64_t ldx,
                                     const float *dY, int64_t lddy, int32_t F, float slope,
                                     const float *alpha, float *d_aL, void *stream) {
    if (!wR && A && A->n_rows > 0) return GALA_ERR_INVALID_ARG;
    return gat_bwd_impl(A, aL, nullptr, wR, bR, X, ldx, dY, lddy, F, 1, slope, GALA_SOFTMAX_REF,
                        alpha, nullptr, d_aL, stream);
}

extern "C" int gala_edge_permute_f32(const int32_t *perm, const float *src, int64_t n,
                                     int32_t heads, float *dst, void *stream) {
    if (n < 0 || heads < 1) return GALA_ERR_INVALID_ARG;
    if (n == 0) return GALA_OK;
    if (!perm || !src || !dst) return GALA_ERR_INVALID_ARG;
    const int64_t total = n * heads;
    const int64_t blocks = (total + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(k_permute, dim3((unsigned)blocks), dim3(kBlock), 0, (hipStream_t)stream,
                       perm, src, n, heads, dst);
    return launch_status();
}
