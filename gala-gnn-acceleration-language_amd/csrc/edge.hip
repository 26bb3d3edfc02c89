// Edge-parallel ops of the GAT pipeline for gfx950: SDDVV (add / mul / add+LeakyReLU),
// edge->row sum, row->edge scale, SDDMM dot, edge-softmax forward/backward and the
// edge-value permutation (the fused GAT kernels are in gat.hip, shared pieces in
// edge_common.h).
//
// Replaces the emitted kernels default_function_kernel_sddvv_{plus,mult}_undir
// (src/codegen/cuda.h:679-698, 848-867), spmm_backward_sddmm_32_{nln,eaggr}
// (505-524, 659-678), {softmax,mult}_sddvv_undir (525-562), sddmm_mult_undir_shared
// (699-734) and the torch compositions around them (src/codegen/common.h:735-810).
//
// Row-segment ops ("RS" kernels): a group of G lanes owns one row and strides over its
// edges (coalesced edge arrays), reductions use xor butterflies inside the group.
#include "edge_common.h"

namespace gala {

// ---- row-segment edge ops over flattened (edge, head) elements ----------------------
// With HP heads (a power of two dividing G) the row's HP*deg edge values are contiguous,
// lane g always handles head g % HP, and per-head reductions run over the xor offsets
// G/2 .. HP.  Non-power-of-two head counts use the *_generic kernels further down.
// (Register tiles: edge_common.h.)

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

// The reference's K7 sum in its own order (cuda.h:505-524: one thread per row, local = eps,
// then local + v[e] for every edge in CSR order): the row group loads a register tile of G*K
// values coalesced (value t of the row slice at lane t mod G, slot t div G), parks it in the
// group's LDS region head-major ([head][value / HP], value t at head t mod HP), and lane
// h < HP adds its head's values in edge order from there with 16-B reads -- the chain waits
// on nothing but its own adds.  Values of the slice are vr[t * stride], t < n (stride > 1:
// one head of an [E, H] array).  Returns the chain in lanes gl < HP (the head of lane gl);
// the other lanes' value is meaningless.  The tile's tail holds +0.0f: adding it is exact
// (local is never -0.0f: it starts at eps >= +0 and x + (-x) rounds to +0).
constexpr int kChainRow = kTileK * kWave;  // floats of one wave's tile
template <int G, int HP>
struct ChainLds {
    static constexpr int per_head = G * kTileK / HP + 4;   // padded: heads on other banks
    static constexpr int per_group = HP * per_head;
    static constexpr int per_wave = (kWave / G) * per_group;
};

template <int G, int HP>
__device__ __forceinline__ float chain_range(const float *vr, int64_t n, int64_t stride, int gl, float local,
                                             float *lg) {
    constexpr int K = kTileK;
    typedef ChainLds<G, HP> L;
    float *mine = lg + (gl & (HP - 1)) * L::per_head;   // this lane's head row (lanes gl < HP chain)
    for (int64_t t0 = 0; t0 < n; t0 += G * K) {
        float x[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {   // clamped: every load is unconditional (n > t0 >= 0)
            const int64_t t = t0 + gl + (int64_t)k * G;
            const float xv = vr[(t < n ? t : n - 1) * stride];
            x[k] = t < n ? xv : 0.0f;
        }
        // value t = k*G + gl -> head t mod HP = gl mod HP, position t div HP
#pragma unroll
        for (int k = 0; k < K; ++k) lg[(gl & (HP - 1)) * L::per_head + k * (G / HP) + gl / HP] = x[k];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (gl < HP) {
            const int64_t rem = n - t0;
            const int cnt = (int)(((rem < G * K ? rem : G * K) + HP - 1) / HP);   // this head's values
            const float4 *q = reinterpret_cast<const float4 *>(mine);
            for (int j = 0; j < cnt; j += 16) {
                float4 a[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) a[i] = (j + 4 * i < cnt) ? q[j / 4 + i] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    local = __fadd_rn(local, a[i].x);
                    local = __fadd_rn(local, a[i].y);
                    local = __fadd_rn(local, a[i].z);
                    local = __fadd_rn(local, a[i].w);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();   // the chain lanes' reads before the next tile's writes
    }
    return local;
}

// K7 for every row in the reference's order: per segment local = eps + the segment's values
// in CSR order, added to the row's running value (segment 0 first; cuda.h:505-524,659-678,
// whose per-segment launches each add one segment's local to C) -- bit-identical.
template <int G, int HP>
__global__ __launch_bounds__(kBlock) void k_row_sum(EdgeParams p, const float *v, float eps,
                                                    int accum, float *out, int32_t thr) {
    typedef ChainLds<G, HP> L;
    __shared__ __attribute__((aligned(16))) float chain_tile[(kBlock / kWave) * L::per_wave];
    GALA_ROW_PROLOGUE(G);
    constexpr int LH = __builtin_ctz(HP);
    if (!row_ok || hub_row(p, thr, row)) return;   // hub rows: k_row_sum_hub / the chunks
    float *lg = chain_tile + (threadIdx.x / kWave) * L::per_wave + (lane / G) * L::per_group;
    float c = (accum && gl < HP) ? out[row * HP + gl] : 0.0f;
    for (int s = 0; s < p.seg.n; ++s) {
        int64_t e0, e1;
        row_range(p, s, row, e0, e1);
        c = __fadd_rn(c, chain_range<G, HP>(v + (e0 << LH), (e1 - e0) << LH, 1, gl, eps, lg));
    }
    if (gl < HP) out[row * HP + gl] = c;
}

// Hub rows of K7 in the reference's order (the default; GALA_SPMM_HUB_CHUNKED selects the
// chunk partials below): one workgroup per (hub row, slice of <= 64 heads).  Waves 1-3 stage
// tile t+1 of the row's values head-major in LDS ([head][edge], double-buffered) while lane h
// of wave 0 adds tile t of its head in edge order -- the serial chain of the reference's
// thread per row, fed from LDS so no global load latency sits in it.
constexpr int kChainBuf = 6144;  // floats of values per LDS buffer
constexpr int kChainPad = 4;     // per-head row padding: heads land on different banks
static_assert(kChainBuf / kWave >= 16, "a tile holds at least 16 edges of every head");

__global__ __launch_bounds__(kBlock) void k_row_sum_hub(EdgeParams p, const float *v, float eps, int accum,
                                                        float *out, HubSplit sp, int32_t n_slices) {
    extern __shared__ __attribute__((aligned(16))) float chain_lds[];
    const int64_t ri = blockIdx.x / n_slices;
    const int h0 = (int)(blockIdx.x % n_slices) * kWave;
    const int H = p.heads;
    const int hs = (H - h0) < kWave ? (H - h0) : kWave;        // heads of this slice (a power of two)
    const int lhs = __builtin_ctz(hs);
    const int TE = (kChainBuf >> lhs) & ~15;                    // edges per tile, a multiple of 16
    const int ld = TE + kChainPad;                              // LDS row of one head
    const int buf_floats = hs * ld;
    const int64_t row = sp.rows[ri];
    const int64_t e0 = p.rowptr[row], n = (int64_t)p.rowptr[row + 1] - e0;
    const int ntiles = (int)((n + TE - 1) / TE);
    const bool chain = threadIdx.x < kWave;
    const int g = threadIdx.x - kWave;
    constexpr int kLoaders = kBlock - kWave;                    // 192: a multiple of every hs
    const int lh = g & (hs - 1), estep = kLoaders >> lhs;
    auto tile_edges = [&](int t) { return (int)((n - (int64_t)t * TE) < TE ? (n - (int64_t)t * TE) : TE); };
    // loader thread g: head g mod hs, edges g / hs + k * (192 / hs) of the tile; the last
    // tile's row tail up to a multiple of 16 is zero-filled (+0.0f adds are exact: local is
    // never -0.0f)
    // (32 loads in flight per thread -- a whole tile in one round trip for every slice width
    // -- clamped to the tile: unconditional)
    auto fill = [&](int t) {
        constexpr int U = 32;
        float *b = chain_lds + (t & 1) * buf_floats + lh * ld;
        const float *src = v + (e0 + (int64_t)t * TE) * H + h0 + lh;
        const int ne = tile_edges(t), ne16 = (ne + 15) & ~15;
        for (int ea = g >> lhs; ea < ne16; ea += U * estep) {
            float x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = ea + u * estep;
                const float xv = src[(int64_t)(e < ne ? e : ne - 1) * H];
                x[u] = e < ne ? xv : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (ea + u * estep < ne16) b[ea + u * estep] = x[u];
        }
    };
    if (!chain) fill(0);
    __syncthreads();
    float local = eps;
    const int lane = threadIdx.x;
    for (int t = 0; t < ntiles; ++t) {
        if (!chain) {
            if (t + 1 < ntiles) fill(t + 1);
        } else if (lane < hs) {
            // groups of 16 values: 4 16-B reads, then 16 dependent adds (8.3 cycles per add
            // measured on the 388 K-edge row; explicit read-ahead, 32- or 64-value groups and
            // s_setprio measured no better, tools/row_sum_probe.py)
            const float *bb = chain_lds + (t & 1) * buf_floats + lane * ld;
            const int n16 = (tile_edges(t) + 15) >> 4;
            for (int i = 0; i < n16; ++i) {
                float4 q[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) q[k] = *reinterpret_cast<const float4 *>(bb + 16 * i + 4 * k);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    local = __fadd_rn(local, q[k].x);
                    local = __fadd_rn(local, q[k].y);
                    local = __fadd_rn(local, q[k].z);
                    local = __fadd_rn(local, q[k].w);
                }
            }
        }
        __syncthreads();
    }
    if (chain && lane < hs) {
        const int64_t o = row * H + h0 + lane;
        out[o] = __fadd_rn(accum ? out[o] : 0.0f, local);
    }
}

static inline size_t row_sum_hub_lds(int heads) {   // heads: a power of two
    const int hs = heads < kWave ? heads : kWave;
    const int TE = (kChainBuf / hs) & ~15;
    return 2 * (size_t)hs * (TE + kChainPad) * sizeof(float);
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
// any head count: one head at a time, each in the reference's order (k_row_sum's chain over
// the head's strided values)
template <int G>
__global__ __launch_bounds__(kBlock) void k_row_sum_generic(EdgeParams p, const float *v, float eps,
                                                    int accum, float *out) {
    typedef ChainLds<G, 1> L;
    __shared__ __attribute__((aligned(16))) float chain_tile[(kBlock / kWave) * L::per_wave];
    GALA_ROW_PROLOGUE(G);
    if (!row_ok) return;
    float *lg = chain_tile + (threadIdx.x / kWave) * L::per_wave + (lane / G) * L::per_group;
    const int H = p.heads;
    for (int h = 0; h < H; ++h) {
        float c = (accum && gl == 0) ? out[row * H + h] : 0.0f;
        for (int s = 0; s < p.seg.n; ++s) {
            int64_t e0, e1;
            row_range(p, s, row, e0, e1);
            c = __fadd_rn(c, chain_range<G, 1>(v + e0 * H + h, e1 - e0, H, gl, eps, lg));
        }
        if (gl == 0) out[row * H + h] = c;
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
template <int M, int O, int U>
__device__ __forceinline__ void reduce_scatter_step(float (&v)[U], int gl) {
    if constexpr (M > 1) {
        const bool up = (gl & O) != 0;
#pragma unroll
        for (int i = 0; i < M / 2; ++i) {
            const float send = up ? v[i] : v[i + M / 2];
            const float keep = up ? v[i + M / 2] : v[i];
            v[i] = keep + lane_xor<O>(send);
        }
        reduce_scatter_step<M / 2, O / 2, U>(v, gl);
    }
}
template <int G, int U>
__device__ __forceinline__ float reduce_scatter(float (&v)[U], int gl) {
    reduce_scatter_step<U, G / 2, U>(v, gl);
    return group_sum<G / U>(v[0]);
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

// edge-value permutation: dst[i, h] = src[perm[i], h] (an edge array into transposed order)
__global__ __launch_bounds__(kBlock) void k_permute(const int32_t *perm, const float *src,
                                                    int64_t n, int32_t H, float *dst) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= n * H) return;
    const int64_t i = t / H;
    const int h = (int)(t % H);
    dst[t] = src[(int64_t)perm[i] * H + h];
}

}  // namespace gala

using namespace gala;

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
    if (flags & ~(GALA_SPMM_ACCUM | GALA_SPMM_HUB_CHUNKED)) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0) return GALA_OK;
    if (!out_row || (!v_e && A->nnz > 0)) return GALA_ERR_INVALID_ARG;
    const int accum = (flags & GALA_SPMM_ACCUM) ? 1 : 0;
    hipStream_t hs = (hipStream_t)stream;
    const int hp = pow2_heads(heads);
    if (hp) {
        const int G = std::max(pick_group_tiled(A, heads), hp);
        const dim3 grid(blocks_for(A->n_rows, G));
        HubSplit sp{};
        const bool chunked = (flags & GALA_SPMM_HUB_CHUNKED) != 0;
        // REF order (default): the hub rows' serial chains; chunked: partials + ordered fix-up
        const bool split = hub_split(A, chunked ? 2 * (int64_t)hp : 0, &sp);
        const int32_t thr = split ? sp.threshold : 0;
        if (split && !chunked) {   // the long chains first, beside the row kernel when the plan has a side stream
            const int ns = (heads + kWave - 1) / kWave;
            HubFork fk(A->split, hs);
            st = fk.fork();
            if (st) return st;
            hipLaunchKernelGGL(k_row_sum_hub, dim3((unsigned)(sp.n_rows_split * ns)), dim3(kBlock),
                               row_sum_hub_lds(heads), fk.side, p, v_e, eps, accum, out_row, sp, ns);
            st = launch_status();
            if (!st) {
                GALA_DISPATCH_GH(G, hipLaunchKernelGGL((k_row_sum<GG, HH>), grid, dim3(kBlock), 0, hs, p, v_e, eps,
                                                       accum, out_row, thr));
                st = launch_status();
            }
            return fk.join(st);
        }
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
    // any other head count: every row (hub rows too) in one sequential pass per head
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
