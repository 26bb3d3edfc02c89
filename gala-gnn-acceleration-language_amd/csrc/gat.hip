// gat.hip -- the fused GAT kernels for gfx950: one pass per row for the forward
// (logits, LeakyReLU, edge softmax, attention-weighted aggregation, alpha out) and for
// the backward edge chain (d alpha, softmax backward, LeakyReLU backward, row sums), with
// hub-row chunk partials, attention recompute (RC) and row-padded operands.
// Replaces the torch compositions around the emitted GAT kernels
// (src/codegen/common.h:622-675, 735-810, 835-894; cuda.h:505-524, 679-734, 808-845).
#include "gat_common.h"

namespace gala {

// ---- fused GAT aggregation -----------------------------------------------------------
// Row group of G lanes, lane g owns CH x VEC features (Lanes); U edges per batch: cols,
// aR[col] and the X row slices are all loaded before the softmax updates.

// Running state of the forward for one row / chunk: per lane CH x VEC accumulators and the
// head's (max, sum) of the softmax (FIXED: online, relative to m; REF: plain sums).
// kRefStats adds the row statistics' sums: accm = sum m*p*X and sma = sum m*p (m the
// LeakyReLU factor of the edge), both scaled by q at the store like acc and sum.
// self_row >= 0 (RC row statistics with ar_out): the column of the row's own vertex; its
// recomputed source logit is captured from the self-loop edge (ar_self, has_self), so the
// vertex's X line is not re-read.
template <int VEC, int CH>
struct FwdState {
    float acc[CH][VEC], accm[CH][VEC];
    float m, sum, sma;
    int64_t self_row;
    float ar_self;
    bool has_self;
    __device__ __forceinline__ FwdState() : m(-INFINITY), sum(0.0f), sma(0.0f), self_row(-1), ar_self(0.0f), has_self(false) {
#pragma unroll
        for (int ch = 0; ch < CH; ++ch)
#pragma unroll
            for (int i = 0; i < VEC; ++i) acc[ch][i] = accm[ch][i] = 0.0f;
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
            if (ref_mode(MODE)) {
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

// The same edges with the per-edge scalar work distributed over the head's HW lanes
// (HW a power of two; HW = G for one head).  The lanes of a head own its features, so the
// old loop repeated each edge's aR load, logit, LeakyReLU and exp on all HW lanes (8.77e9
// -> 18.2e9 VALU instructions against the weighted SpMM at 8 heads).  Here edge k of a
// U-edge batch is worked by lane k mod HW of the head group (its aR load, logit and exp),
// and its exp term is broadcast to the group for the accumulation, which stays sequential
// in CSR order (REF: bit-identical results to the per-lane loop).  The same lanes park the
// terms in the alpha buffer: one coalesced (edge, head) store per batch.  FIXED mode takes
// the batch's max over the group first and rescales the running state once per batch.
template <int G, int VEC, int U, int MODE, int CH, bool RC, int HW>
__device__ __forceinline__ void gat_fwd_range_dist(const EdgeParams &p, const GatDev &d,
                                                   const GatLane<G, VEC, CH, RC> &gl_, bool park,
                                                   int64_t e0, int64_t e1, FwdState<VEC, CH> &st) {
    typedef typename GVec<VEC>::T V;
    constexpr int UH = (U < HW) ? U : HW;  // distinct edge owners per head group
    constexpr int NK = U / UH;              // edges per owner lane
    const int H = gl_.H, hh = gl_.hh;
    const int lane = threadIdx.x & (kWave - 1);
    const int hl = lane & (HW - 1);
    const int kl = hl % UH;                // this lane's first edge of a batch
    // owners hold their head's values: every lane for one head, valid lanes for several
    const bool store = park && hl < UH && (H == 1 || gl_.cv);
    const int32_t n = (int32_t)(e1 - e0);
    // The parked terms of a batch are stored one batch late, after the next batch's loads
    // are issued: stores count in vmcnt, and a store issued ahead of the loads made every
    // batch wait out its write latency (8 heads: 3 ms over the no-alpha forward).
    float pend[NK];
    int32_t pend_j0 = -1;
    int32_t win = 0;  // the row's next 64 column indices (load_batch_cols_win)
    for (int32_t j0 = 0; j0 < n; j0 += U) {
        int64_t c[U];
        V x[U][CH];
        load_batch_cols_win<G, U>(p, e0, n, j0, win, c);
        float ar[NK];
        if (!RC) {
#pragma unroll
            for (int i = 0; i < NK; ++i) {
                const int32_t j = (j0 + kl + i * UH < n) ? j0 + kl + i * UH : n - 1;
                ar[i] = d.aR[(int64_t)p.col[e0 + j] * H + hh];
            }
        }
        // given source logits: the X rows are loaded nontemporal, so the gathered rows do not
        // evict the aR table every edge also reads a line of (one head, F = 32, the Products
        // graph: 4.31 -> 3.87 ms in one process, tools/ab_gat.py h1f32).  Recomputed logits
        // read no such table, and there the hint only costs the rows' reuse.
#pragma unroll
        for (int k = 0; k < U; ++k)
#pragma unroll
            for (int ch = 0; ch < CH; ++ch) {
                const V *xp = reinterpret_cast<const V *>(d.X + c[k] * d.ldx + gl_.ln.off[ch]);
                x[k][ch] = mask_pad<VEC>(gl_.ln.nv[ch], RC ? *xp : __builtin_nontemporal_load(xp));
            }
        if (store && pend_j0 >= 0) {
#pragma unroll
            for (int i = 0; i < NK; ++i)  // a previous batch is always full
                d.alpha_out[(e0 + pend_j0 + kl + i * UH) * H + hh] = pend[i];
        }
        if (RC) {  // the U source logits from the gathered rows (every lane of the head gets all)
            float all[U];
#pragma unroll
            for (int k = 0; k < U; ++k) all[k] = __fadd_rn(attn_dot<HW, VEC, CH>(gl_.w, x[k]), gl_.wb);
            if constexpr (MODE == kRefStats) {
                // the self-loop edge's logit is the row's own aR: the same gathered row, lanes,
                // fma order and butterfly as the X[row] recompute it replaces (bit-identical)
                if (st.self_row >= 0) {
#pragma unroll
                    for (int k = 0; k < U; ++k)
                        if (j0 + k < n && c[k] == st.self_row) {
                            st.ar_self = all[k];
                            st.has_self = true;
                        }
                }
            }
#pragma unroll
            for (int i = 0; i < NK; ++i) {
                float v = all[0];
#pragma unroll
                for (int k = 1; k < U; ++k) v = (kl + i * UH == k) ? all[k] : v;
                ar[i] = v;
            }
        }
        float pe[NK], z[NK];
        bool pos[NK];
#pragma unroll
        for (int i = 0; i < NK; ++i) {
            float t = __fadd_rn(gl_.al, ar[i]);
            pos[i] = t > 0.0f;
            z[i] = pos[i] ? t : __fmul_rn(t, d.slope);
        }
        if (ref_mode(MODE)) {
#pragma unroll
            for (int i = 0; i < NK; ++i) pe[i] = ref_exp(z[i]);
        } else {
            float mb = -INFINITY;
#pragma unroll
            for (int i = 0; i < NK; ++i) mb = (j0 + kl + i * UH < n) ? fmaxf(mb, z[i]) : mb;
            mb = group_max<HW>(mb);
            if (mb > st.m) {
                const float r = (st.m == -INFINITY) ? 0.0f : expf(st.m - mb);
                st.sum = __fmul_rn(st.sum, r);
#pragma unroll
                for (int ch = 0; ch < CH; ++ch)
#pragma unroll
                    for (int i = 0; i < VEC; ++i) st.acc[ch][i] = __fmul_rn(st.acc[ch][i], r);
                st.m = mb;
            }
#pragma unroll
            for (int i = 0; i < NK; ++i) pe[i] = expf(z[i] - st.m);
        }
        if (store) {
#pragma unroll
            for (int i = 0; i < NK; ++i) pend[i] = (ref_mode(MODE)) ? pe[i] : z[i];
            pend_j0 = j0;
        }
        float mp[NK];  // kRefStats: m * p, m = 1 on the LeakyReLU's positive side, else slope
        if constexpr (MODE == kRefStats) {
#pragma unroll
            for (int i = 0; i < NK; ++i) mp[i] = pos[i] ? pe[i] : __fmul_rn(pe[i], d.slope);
        }
        static_for<0, U>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            const float pk = group_bcast<HW, k % UH>(pe[k / UH]);
            float mk = 0.0f;
            if constexpr (MODE == kRefStats) mk = group_bcast<HW, k % UH>(mp[k / UH]);
            if (j0 + k >= n) return;
            st.sum = __fadd_rn(st.sum, pk);
#pragma unroll
            for (int ch = 0; ch < CH; ++ch) {
                const float *xv = reinterpret_cast<const float *>(&x[k][ch]);
#pragma unroll
                for (int i = 0; i < VEC; ++i) st.acc[ch][i] = fmaf(pk, xv[i], st.acc[ch][i]);
            }
            if constexpr (MODE == kRefStats) {
                st.sma = __fadd_rn(st.sma, mk);
#pragma unroll
                for (int ch = 0; ch < CH; ++ch) {
                    const float *xv = reinterpret_cast<const float *>(&x[k][ch]);
#pragma unroll
                    for (int i = 0; i < VEC; ++i) st.accm[ch][i] = fmaf(mk, xv[i], st.accm[ch][i]);
                }
            }
        });
    }
    if (store && pend_j0 >= 0) {
#pragma unroll
        for (int i = 0; i < NK; ++i)
            if (pend_j0 + kl + i * UH < n) d.alpha_out[(e0 + pend_j0 + kl + i * UH) * H + hh] = pend[i];
    }
}

template <int G, int VEC, int U, int MODE, int CH, bool RC, int HW>
__device__ __forceinline__ void gat_fwd_edges(const EdgeParams &p, const GatDev &d,
                                              const GatLane<G, VEC, CH, RC> &gl_, bool park,
                                              int64_t e0, int64_t e1, FwdState<VEC, CH> &st) {
    if constexpr (HW > 0)
        gat_fwd_range_dist<G, VEC, U, MODE, CH, RC, HW>(p, d, gl_, park, e0, e1, st);
    else
        gat_fwd_range<G, VEC, U, MODE, CH, RC>(p, d, gl_, park, e0, e1, st);
}

// A continuation's starting state (d.init_acc set, REF): the row's partials of the earlier pass.
template <int G, int VEC, int CH, bool RC, int MODE>
__device__ __forceinline__ void gat_fwd_init(const GatDev &d, const GatLane<G, VEC, CH, RC> &gl_, int64_t row,
                                             FwdState<VEC, CH> &st) {
    typedef typename GVec<VEC>::T V;
    if (!d.init_acc) return;
    auto load = [&](const float *base, int64_t ld, float (&dst)[CH][VEC]) {
#pragma unroll
        for (int ch = 0; ch < CH; ++ch) {
            if (!gl_.ln.valid[ch]) continue;
            const float *src = base + row * ld + gl_.ln.off[ch];
            if (gl_.ln.nv[ch] == VEC) {
                const V v = *reinterpret_cast<const V *>(src);
                const float *vv = reinterpret_cast<const float *>(&v);
#pragma unroll
                for (int i = 0; i < VEC; ++i) dst[ch][i] = vv[i];
            } else {
#pragma unroll
                for (int i = 0; i < VEC; ++i)
                    if (gl_.ln.in(ch, i)) dst[ch][i] = src[i];
            }
        }
    };
    load(d.init_acc, d.ld_init, st.acc);
    if (gl_.cv) st.sum = d.init_sum[row * gl_.H + gl_.hh];
    if constexpr (MODE == kRefStats) {
        load(d.init_accm, d.ld_initm, st.accm);
        if (gl_.cv) st.sma = d.init_sma[row * gl_.H + gl_.hh];
    }
}

// Y[row] = acc * q with q = 1 / (sum [+ S * 1e-12 in REF mode]); returns q.  Partial
// (GALA_GAT_PARTIAL, REF): Y = acc unnormalised and the raw sum is returned, for a caller
// that adds the partial rows of several column ranges first (vertex cut).
template <int G, int VEC, int CH, bool RC, int MODE>
__device__ __forceinline__ float gat_fwd_store(const GatDev &d, const GatLane<G, VEC, CH, RC> &gl_,
                                               int64_t row, int nseg, const FwdState<VEC, CH> &st) {
    typedef typename GVec<VEC>::T V;
    const float den = (ref_mode(MODE)) ? st.sum + (float)nseg * 1e-12f : st.sum;
    const float q = d.partial ? 1.0f : 1.0f / den;
#pragma unroll
    for (int ch = 0; ch < CH; ++ch) {
        if (!gl_.ln.valid[ch]) continue;
        V out;
        float *ov = reinterpret_cast<float *>(&out);
#pragma unroll
        for (int i = 0; i < VEC; ++i)
            ov[i] = d.partial ? st.acc[ch][i]
                    : (!ref_mode(MODE) && st.sum == 0.0f) ? 0.0f : __fmul_rn(st.acc[ch][i], q);
        float *yp = d.Y + row * d.ldy + gl_.ln.off[ch];
        if (gl_.ln.nv[ch] == VEC) {
            *reinterpret_cast<V *>(yp) = out;
        } else {  // a padded row's last vector: its real columns only
#pragma unroll
            for (int i = 0; i < VEC; ++i)
                if (gl_.ln.in(ch, i)) yp[i] = ov[i];
        }
        if constexpr (MODE == kRefStats) {
#pragma unroll
            for (int i = 0; i < VEC; ++i) ov[i] = __fmul_rn(st.accm[ch][i], q);
            float *mp = d.ym_out + row * d.ldym + gl_.ln.off[ch];
            if (gl_.ln.nv[ch] == VEC) {
                *reinterpret_cast<V *>(mp) = out;
            } else {
#pragma unroll
                for (int i = 0; i < VEC; ++i)
                    if (gl_.ln.in(ch, i)) mp[i] = ov[i];
            }
        }
    }
    if constexpr (MODE == kRefStats)
        if (gl_.leader) d.sma_out[row * gl_.H + gl_.hh] = __fmul_rn(st.sma, q);
    return d.partial ? st.sum : q;
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
            const float pe = (ref_mode(MODE)) ? v[k] : expf(v[k] - mh);
            if (t < n) ar[t] = __fmul_rn(pe, qh);
        }
    }
}

// One pass per row: logits, LeakyReLU, softmax (REF exp-clamp / FIXED online max), the
// alpha-weighted aggregation, then 1/sum; alpha (if requested) in a parked-value pass.
template <int G, int VEC, int U, int MODE, int CH, bool RC, int HW>
__global__ __launch_bounds__(kBlock) void k_gat_fwd(EdgeParams p, GatDev d, int32_t split_threshold) {
    GALA_ROW_PROLOGUE(G);
    if (!row_ok) return;
    const GatLane<G, VEC, CH, RC> gl_(p, d, gl, row);
    constexpr bool kArOut = RC && MODE == kRefStats && HW > 0;
    // the own vertex's source logit for the backward's alpha, formed exactly as the per-edge
    // recompute forms it (same lanes, same fma order and butterfly): taken from the row's
    // self-loop edge when it has one (every GALA graph does, gala_export_npy.py:73-74),
    // else (and for hub rows, whose edges the chunk kernels walk) from a read of X[own].
    // The own vertex is the row itself on one GPU, self_col[row] over a vertex cut (whose
    // rows are destinations and whose columns are the rank's vertices).
    const int64_t own = !kArOut || !d.ar_out ? -1 : d.self_col ? (int64_t)d.self_col[row] : row;
    auto ar_of_own = [&]() {
        typedef typename GVec<VEC>::T V;
        V xr[CH];
#pragma unroll
        for (int ch = 0; ch < CH; ++ch)
            xr[ch] = mask_pad<VEC>(gl_.ln.nv[ch], *reinterpret_cast<const V *>(d.X + own * d.ldx + gl_.ln.off[ch]));
        return __fadd_rn(attn_dot<HW, VEC, CH>(gl_.w, xr), gl_.wb);
    };
    const bool hub = split_threshold > 0 && p.rowptr[row + 1] - p.rowptr[row] > split_threshold;
    if constexpr (kArOut) {
        if (own >= 0 && hub) {
            const float a = ar_of_own();
            if (gl_.leader) d.ar_out[own * gl_.H + gl_.hh] = a;
        }
    }
    if (hub) return;  // hub row: k_gat_fwd_chunk / _fixup / k_gat_alpha_chunk
    const int H = gl_.H, D = gl_.D;
    // With H | G the main pass parks each (edge, head)'s exp term (REF) or logit (FIXED)
    // in alpha_out (the head's first lane writes it) and the alpha pass rescales it in
    // place: a contiguous re-read of the row instead of a second col -> aR gather.
    const bool park = d.alpha_out != nullptr && (G % H) == 0;
    FwdState<VEC, CH> st;
    if constexpr (ref_mode(MODE)) gat_fwd_init<G, VEC, CH, RC, MODE>(d, gl_, row, st);
    if constexpr (kArOut) st.self_row = own;
    for (int s = 0; s < p.seg.n; ++s) {
        int64_t e0, e1;
        row_range(p, s, row, e0, e1);
        gat_fwd_edges<G, VEC, U, MODE, CH, RC, HW>(p, d, gl_, park, e0, e1, st);
    }
    if constexpr (kArOut) {
        if (own >= 0) {
            const float a = st.has_self ? st.ar_self : ar_of_own();
            if (gl_.leader) d.ar_out[own * gl_.H + gl_.hh] = a;
        }
    }
    const float q = gat_fwd_store<G, VEC, CH, RC, MODE>(d, gl_, row, p.seg.n, st);
    if (d.q_out && gl_.leader) d.q_out[row * H + gl_.hh] = q;  // factored: alpha = p * q
    if (!d.alpha_out) return;
    const int gbase = (threadIdx.x & (kWave - 1)) & ~(G - 1);
    if (park) {
        if (d.q_out) return;  // the parked exp terms are the output
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
                const float pe = (ref_mode(MODE)) ? ref_exp(z) : expf(z - mh);
                d.alpha_out[e * H + hd] = d.q_out ? pe : __fmul_rn(pe, qh);
            }
        }
    }
}


// hub rows, forward: chunk partial state -> ws[c] = {acc[F], m[H], sum[H]}
template <int G, int VEC, int U, int MODE, int CH, bool RC, int HW>
__global__ __launch_bounds__(kBlock) void k_gat_fwd_chunk(EdgeParams p, GatDev d, HubSplit sp) {
    GALA_CHUNK_PROLOGUE(G);
    const GatLane<G, VEC, CH, RC> gl_(p, d, gl, row);
    FwdState<VEC, CH> st;
    gat_fwd_edges<G, VEC, U, MODE, CH, RC, HW>(p, d, gl_, d.alpha_out != nullptr, e0, e1, st);
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
    if constexpr (MODE == kRefStats) {  // ws[c] continues {accm[F], sma[H]}
        float *wm = w + d.F + 2 * gl_.H;
#pragma unroll
        for (int ch = 0; ch < CH; ++ch)
#pragma unroll
            for (int i = 0; i < VEC; ++i)
                if (gl_.ln.in(ch, i)) wm[gl_.ln.off[ch] + i] = st.accm[ch][i];
        if (gl_.leader) wm[d.F + gl_.hh] = st.sma;
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
    if constexpr (ref_mode(MODE)) gat_fwd_init<G, VEC, CH, RC, MODE>(d, gl_, row, st);
    const int64_t c0 = sp.row_chunk0[ri], c1 = sp.row_chunk0[ri + 1];
    for (int64_t cc = c0; cc < c1; ++cc) {
        const float *w = sp.ws + cc * sp.ws_cols;
        const float mc = w[F + hh], sc = w[F + H + hh];
        float a = 1.0f, b = 1.0f;
        if (!ref_mode(MODE)) {
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
                st.acc[ch][i] = (ref_mode(MODE)) ? __fadd_rn(st.acc[ch][i], v)
                                                           : fmaf(st.acc[ch][i], a, __fmul_rn(v, b));
            }
        if constexpr (MODE == kRefStats) {
            const float *wm = w + F + 2 * H;
            st.sma = __fadd_rn(st.sma, wm[F + hh]);
#pragma unroll
            for (int ch = 0; ch < CH; ++ch)
#pragma unroll
                for (int i = 0; i < VEC; ++i)
                    st.accm[ch][i] = __fadd_rn(st.accm[ch][i], gl_.ln.in(ch, i) ? wm[gl_.ln.off[ch] + i] : 0.0f);
        }
    }
    const float q = gat_fwd_store<G, VEC, CH, RC, MODE>(d, gl_, row, 1, st);
    if (gl_.leader && d.q_out) {
        d.q_out[row * H + hh] = q;
    } else if (gl_.leader && d.alpha_out) {
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
        if (d.q) {  // factored attention (p, q): alpha = p * q, rounded as materialised
#pragma unroll
            for (int k = 0; k < U; ++k) a[k] = __fmul_rn(a[k], gl_.qr);
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
            for (int k = 0; k < U; ++k) ar[k] = __fadd_rn(attn_dot<HW, VEC, CH>(gl_.w, x[k]), gl_.wb);
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

}  // namespace gala

using namespace gala;

// Host-side launch description of the fused GAT kernels (forward and backward).
struct GatArgs {
    EdgeParams p;
    GatDev d;
    HubSplit sp;
    bool split;
    int mode;
    hipStream_t hs;
};


template <int G, int VEC, int CH, bool RC, int HW, int MODE>
static void launch_gat_mode(const GatArgs &a) {
    constexpr int U = 8;
    hipLaunchKernelGGL((k_gat_fwd<G, VEC, U, MODE, CH, RC, HW>), dim3(blocks_for(a.p.n_rows, G)), dim3(kBlock),
                       0, a.hs, a.p, a.d, a.split ? a.sp.threshold : 0);
    if (!a.split) return;
    hipLaunchKernelGGL((k_gat_fwd_chunk<G, VEC, U, MODE, CH, RC, HW>), dim3(blocks_for_groups(a.sp.n_chunks, G)),
                       dim3(kBlock), 0, a.hs, a.p, a.d, a.sp);
    hipLaunchKernelGGL((k_gat_fwd_fixup<G, VEC, MODE, CH, RC>), dim3(blocks_for_groups(a.sp.n_rows_split, G)),
                       dim3(kBlock), 0, a.hs, a.p, a.d, a.sp);
    if (a.d.alpha_out && !a.d.q_out)
        hipLaunchKernelGGL((k_gat_alpha_chunk<G, VEC, MODE>), dim3(blocks_for_groups(a.sp.n_chunks, G)),
                           dim3(kBlock), 0, a.hs, a.p, a.d, a.sp);
}

template <int G, int VEC, int CH, bool RC, int HW>
static void launch_gat(const GatArgs &a) {
    if (a.mode == kRefStats) {  // row statistics: the head-distributed loop only (HW > 0)
        if constexpr (HW > 0) launch_gat_mode<G, VEC, CH, RC, HW, kRefStats>(a);
        return;
    }
    if (a.mode == GALA_SOFTMAX_REF) launch_gat_mode<G, VEC, CH, RC, HW, GALA_SOFTMAX_REF>(a);
    else launch_gat_mode<G, VEC, CH, RC, HW, GALA_SOFTMAX_FIXED>(a);
}

// several heads: HW = D / VEC lanes per head (a power of two below G) distribute the
// per-edge softmax work; other head widths take the per-lane loop (HW = 0, no RC)
template <int G, int VEC, bool RC>
static int launch_gat_heads(const GatArgs &a, int hw) {
    if constexpr (G >= 2) {
        switch (hw) {
            case 1: launch_gat<G, VEC, 1, RC, 1>(a); return GALA_OK;
            case 2: if constexpr (G > 2) { launch_gat<G, VEC, 1, RC, 2>(a); return GALA_OK; } break;
            case 4: if constexpr (G > 4) { launch_gat<G, VEC, 1, RC, 4>(a); return GALA_OK; } break;
            case 8: if constexpr (G > 8) { launch_gat<G, VEC, 1, RC, 8>(a); return GALA_OK; } break;
            case 16: if constexpr (G > 16) { launch_gat<G, VEC, 1, RC, 16>(a); return GALA_OK; } break;
            case 32: if constexpr (G > 32) { launch_gat<G, VEC, 1, RC, 32>(a); return GALA_OK; } break;
            default: break;
        }
    }
    if (RC || a.mode == kRefStats) return GALA_ERR_UNSUPPORTED;
    launch_gat<G, VEC, 1, false, 0>(a);
    return GALA_OK;
}

template <int G, int VEC, bool RC>
static int launch_gat_g(const GatArgs &a, int heads, int hw) {
    if (heads == 1) {
        launch_gat<G, VEC, 1, RC, G>(a);
        return GALA_OK;
    }
    return launch_gat_heads<G, VEC, RC>(a, hw);
}

template <int VEC, bool RC>
static int gat_vec(const GatArgs &a, int L, int ch, int heads, int hw) {
    if (ch == 2) launch_gat<16, VEC, 2, RC, 16>(a);
    else if (ch == 3) launch_gat<16, VEC, 3, RC, 16>(a);
    else if (ch == 4) launch_gat<16, VEC, 4, RC, 16>(a);
    else if (L <= 1) launch_gat<1, VEC, 1, RC, 1>(a);
    else if (L <= 2) return launch_gat_g<2, VEC, RC>(a, heads, hw);
    else if (L <= 4) return launch_gat_g<4, VEC, RC>(a, heads, hw);
    else if (L <= 8) return launch_gat_g<8, VEC, RC>(a, heads, hw);
    else if (L <= 16) return launch_gat_g<16, VEC, RC>(a, heads, hw);
    else if (L <= 32) return launch_gat_g<32, VEC, RC>(a, heads, hw);
    else if (L <= 64) return launch_gat_g<64, VEC, RC>(a, heads, hw);
    else return GALA_ERR_UNSUPPORTED;
    return GALA_OK;
}


static int gat_fwd_impl(const gala_csr_t *A, const float *aL, const float *aR, const float *wR,
                        const float *bR, const float *X, int64_t ldx, int32_t F, int32_t heads,
                        float slope, int32_t mode, float *Y, int64_t ldy, float *alpha_out,
                        float *q_out, void *stream, float *ym = nullptr, int64_t ldym = 0,
                        float *sma = nullptr, float *ar_out = nullptr, const int32_t *self_col = nullptr,
                        const float *init_acc = nullptr, int64_t ld_init = 0, const float *init_sum = nullptr,
                        const float *init_accm = nullptr, int64_t ld_initm = 0,
                        const float *init_sma = nullptr) {
    GatArgs a{};
    int st = edge_setup(A, heads, &a.p);
    if (st) return st;
    const bool partial = (mode & GALA_GAT_PARTIAL) != 0;
    const bool stats = ym != nullptr;
    mode &= ~GALA_GAT_PARTIAL;
    if (mode != GALA_SOFTMAX_REF && mode != GALA_SOFTMAX_FIXED) return GALA_ERR_INVALID_ARG;
    if (F < 1 || F % heads != 0 || ldx < F || ldy < F || (stats && ldym < F)) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0) return GALA_OK;
    if (!aL || (!aR && !wR) || !Y || (!X && A->nnz > 0)) return GALA_ERR_INVALID_ARG;
    if (q_out && mode != GALA_SOFTMAX_REF) return GALA_ERR_INVALID_ARG;
    if (partial && (mode != GALA_SOFTMAX_REF || !q_out || alpha_out)) return GALA_ERR_INVALID_ARG;
    if (stats && (mode != GALA_SOFTMAX_REF || !q_out || !sma)) return GALA_ERR_INVALID_ARG;
    // a partial pattern's rows are not its columns: aR_out needs the own-vertex map
    if (stats && partial && (alpha_out || (ar_out && !self_col))) return GALA_ERR_INVALID_ARG;
    // square pattern (the backward's dY[col] / aR_out of the row's own X) unless self_col
    // maps each row to its own column (a halo table); a vertex cut's partial forward reads
    // X by column only
    if (stats && !partial && !self_col && !init_acc && A->n_cols > A->n_rows && A->nnz > 0)
        return GALA_ERR_INVALID_ARG;
    if (ar_out && (!stats || aR || !X)) return GALA_ERR_INVALID_ARG;
    // a continuation: REF, no alpha; the statistics need their two partials too
    if (init_acc && (mode != GALA_SOFTMAX_REF || alpha_out || ar_out || !init_sum || ld_init < F ||
                     (stats && (!init_accm || !init_sma || ld_initm < F)) || (!stats && (init_accm || init_sma))))
        return GALA_ERR_INVALID_ARG;
    const int D = F / heads;
    // VEC divides D, or (one head) fits padded rows: ldx, ldy >= F rounded up to VEC
    auto vec_ok = [&](int v) {
        const bool fits = D % v == 0 || (heads == 1 && ldx >= pad_to(F, v) && ldy >= pad_to(F, v) &&
                                         (!stats || ldym >= pad_to(F, v)));
        return fits && ldx % v == 0 && ldy % v == 0 && ((uintptr_t)X % (4 * v)) == 0 &&
               ((uintptr_t)Y % (4 * v)) == 0 && (!stats || (ldym % v == 0 && ((uintptr_t)ym % (4 * v)) == 0)) &&
               (!init_acc || (ld_init % v == 0 && ((uintptr_t)init_acc % (4 * v)) == 0)) &&
               (!init_accm || (ld_initm % v == 0 && ((uintptr_t)init_accm % (4 * v)) == 0));
    };
    int vec = 4;
    while (vec > 1 && !vec_ok(vec)) vec >>= 1;
    const int L = (F + vec - 1) / vec;
    const int ch = narrow_chunks(heads, vec, L);
    int G = 16;
    if (ch == 1) {
        G = 1;
        while (G < L) G <<= 1;
    }
    a.mode = stats ? kRefStats : mode;
    a.d.aL = aL, a.d.aR = aR, a.d.wR = wR, a.d.bR = bR, a.d.X = X, a.d.ldx = ldx, a.d.F = F;
    a.d.slope = slope, a.d.Y = Y, a.d.ldy = ldy, a.d.alpha_out = alpha_out, a.d.q_out = q_out;
    a.d.partial = partial ? 1 : 0;
    a.d.ym_out = ym, a.d.ldym = ldym, a.d.sma_out = sma, a.d.ar_out = ar_out, a.d.self_col = self_col;
    a.d.init_acc = init_acc, a.d.ld_init = ld_init, a.d.init_sum = init_sum;
    a.d.init_accm = init_accm, a.d.ld_initm = ld_initm, a.d.init_sma = init_sma;
    a.hs = (hipStream_t)stream;
    // hub-row chunk partials: {acc[F], m[H], sum[H]} (+ {accm[F], sma[H]} with the statistics)
    const int64_t ws_need = stats ? 2 * (int64_t)F + 3 * heads : (int64_t)F + 2 * heads;
    a.split = (!alpha_out || G % heads == 0) && hub_split(A, ws_need, &a.sp);
    const bool rc = aR == nullptr;
    // alpha of heads that do not divide the row group is formed by a per-head pass that
    // re-reads aR: there is none to read when it is recomputed
    if (rc && alpha_out && G % heads != 0) return GALA_ERR_UNSUPPORTED;
    const int hw = (D % vec == 0) ? D / vec : 0;  // lanes per head (several heads)
    int r;
    if (vec == 4) r = rc ? gat_vec<4, true>(a, L, ch, heads, hw) : gat_vec<4, false>(a, L, ch, heads, hw);
    else if (vec == 2) r = rc ? gat_vec<2, true>(a, L, ch, heads, hw) : gat_vec<2, false>(a, L, ch, heads, hw);
    else r = rc ? gat_vec<1, true>(a, L, ch, heads, hw) : gat_vec<1, false>(a, L, ch, heads, hw);
    if (r) return r;
    return launch_status();
}

extern "C" int gala_gat_fwd_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                const float *X, int64_t ldx, int32_t F, int32_t heads,
                                float slope, int32_t mode, float *Y, int64_t ldy,
                                float *alpha_out, void *stream) {
    if (!aR && A && A->n_rows > 0) return GALA_ERR_INVALID_ARG;
    return gat_fwd_impl(A, aL, aR, nullptr, nullptr, X, ldx, F, heads, slope, mode, Y, ldy,
                        alpha_out, nullptr, stream);
}

extern "C" int gala_gat_fwd_ex_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                   const float *wR, const float *bR, const float *X, int64_t ldx,
                                   int32_t F, int32_t heads, float slope, int32_t mode, float *Y,
                                   int64_t ldy, float *alpha_out, float *q_out, void *stream) {
    if (!aR && !wR && A && A->n_rows > 0) return GALA_ERR_INVALID_ARG;
    return gat_fwd_impl(A, aL, aR, aR ? nullptr : wR, aR ? nullptr : bR, X, ldx, F, heads, slope, mode,
                        Y, ldy, alpha_out, q_out, stream);
}

extern "C" int gala_gat_fwd_stats_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                      const float *wR, const float *bR, const float *X, int64_t ldx,
                                      int32_t F, int32_t heads, float slope, float *Y, int64_t ldy,
                                      float *q_out, float *Ym, int64_t ldym, float *sma, float *aR_out,
                                      float *p_out, void *stream) {
    if (!aR && !wR && A && A->n_rows > 0) return GALA_ERR_INVALID_ARG;
    if (!Ym && A && A->n_rows > 0) return GALA_ERR_INVALID_ARG;
    return gat_fwd_impl(A, aL, aR, aR ? nullptr : wR, aR ? nullptr : bR, X, ldx, F, heads, slope,
                        GALA_SOFTMAX_REF, Y, ldy, p_out, q_out, stream, Ym, ldym, sma, aR_out);
}

// The statistics forward over a gathered table (a row partition's halo): row r's own vertex
// is column self_col[r], which lets the pattern be rectangular; aR_out is column-indexed.
extern "C" int gala_gat_fwd_stats_ex_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                         const float *wR, const float *bR, const float *X, int64_t ldx,
                                         int32_t F, int32_t heads, float slope, float *Y, int64_t ldy,
                                         float *q_out, float *Ym, int64_t ldym, float *sma,
                                         const int32_t *self_col, float *aR_out, float *p_out, void *stream) {
    if (!aR && !wR && A && A->n_rows > 0) return GALA_ERR_INVALID_ARG;
    if (!Ym && A && A->n_rows > 0) return GALA_ERR_INVALID_ARG;
    return gat_fwd_impl(A, aL, aR, aR ? nullptr : wR, aR ? nullptr : bR, X, ldx, F, heads, slope,
                        GALA_SOFTMAX_REF, Y, ldy, p_out, q_out, stream, Ym, ldym, sma, aR_out, self_col);
}

// The row-statistics forward over one column range of a vertex cut: every output unnormalised
// (gat_fwd_store with d.partial), so the owners of the rows add the ranks' partials first.
extern "C" int gala_gat_fwd_partial_stats_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                              const float *wR, const float *bR, const float *X,
                                              int64_t ldx, int32_t F, int32_t heads, float slope, float *U,
                                              int64_t ldu, float *sums, float *Um, int64_t ldum,
                                              float *msums, void *stream) {
    if (!aR && !wR && A && A->n_rows > 0) return GALA_ERR_INVALID_ARG;
    if ((!Um || !sums || !msums) && A && A->n_rows > 0) return GALA_ERR_INVALID_ARG;
    return gat_fwd_impl(A, aL, aR, aR ? nullptr : wR, aR ? nullptr : bR, X, ldx, F, heads, slope,
                        GALA_SOFTMAX_REF | GALA_GAT_PARTIAL, U, ldu, nullptr, sums, stream, Um, ldum, msums,
                        nullptr);
}

// The same with the rank's own vertices' recomputed source logits: row r's own vertex is
// column self_col[r] (-1: none); aR_out[self_col[r] * heads + h] is written bit-identical to
// the logit the kernel forms for that column's edges (the backward's alpha then matches).
extern "C" int gala_gat_fwd_partial_stats_ex_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                                 const float *wR, const float *bR, const float *X,
                                                 int64_t ldx, int32_t F, int32_t heads, float slope, float *U,
                                                 int64_t ldu, float *sums, float *Um, int64_t ldum,
                                                 float *msums, const int32_t *self_col, float *aR_out,
                                                 void *stream) {
    if (!aR && !wR && A && A->n_rows > 0) return GALA_ERR_INVALID_ARG;
    if ((!Um || !sums || !msums) && A && A->n_rows > 0) return GALA_ERR_INVALID_ARG;
    if (aR_out && !self_col) return GALA_ERR_INVALID_ARG;
    return gat_fwd_impl(A, aL, aR, aR ? nullptr : wR, aR ? nullptr : bR, X, ldx, F, heads, slope,
                        GALA_SOFTMAX_REF | GALA_GAT_PARTIAL, U, ldu, nullptr, sums, stream, Um, ldum, msums,
                        aR_out, self_col);
}

// The REF forward continued from an earlier pass's partials over other columns (a row
// partition's own columns while the halo is in flight): Y = q (U0 + sum p X) with
// q = 1 / (S0 + sum p + 1e-12); with Ym the row statistics likewise from (Um0, M0).
// flags GALA_GAT_PARTIAL: the sums continued but left unnormalised (q_out = the raw sum),
// for a further range (a halo arriving in chunks).
extern "C" int gala_gat_fwd_continue_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                         const float *wR, const float *bR, const float *X, int64_t ldx,
                                         int32_t F, int32_t heads, float slope, int32_t flags,
                                         const float *U0, int64_t ldu0,
                                         const float *S0, const float *Um0, int64_t ldum0, const float *M0,
                                         float *Y, int64_t ldy, float *q_out, float *Ym, int64_t ldym,
                                         float *sma, void *stream) {
    if (!aR && !wR && A && A->n_rows > 0) return GALA_ERR_INVALID_ARG;
    if ((!U0 || !S0) && A && A->n_rows > 0) return GALA_ERR_INVALID_ARG;
    if ((Ym != nullptr) != (Um0 != nullptr) || (flags & ~GALA_GAT_PARTIAL) != 0) return GALA_ERR_INVALID_ARG;
    return gat_fwd_impl(A, aL, aR, aR ? nullptr : wR, aR ? nullptr : bR, X, ldx, F, heads, slope,
                        GALA_SOFTMAX_REF | flags, Y, ldy, nullptr, q_out, stream, Ym, ldym, sma, nullptr, nullptr,
                        U0, ldu0, S0, Um0, ldum0, M0);
}

extern "C" int gala_gat_fwd_attn_f32(const gala_csr_t *A, const float *aL, const float *wR,
                                     const float *bR, const float *X, int64_t ldx, int32_t F,
                                     float slope, int32_t mode, float *Y, int64_t ldy,
                                     float *alpha_out, void *stream) {
    if (!wR && A && A->n_rows > 0) return GALA_ERR_INVALID_ARG;
    return gat_fwd_impl(A, aL, nullptr, wR, bR, X, ldx, F, 1, slope, mode, Y, ldy, alpha_out,
                        nullptr, stream);
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
                        const float *alpha, const float *q, float *d_logit, float *d_aL,
                        void *stream) {
    GatArgs a{};
    int st = edge_setup(A, heads, &a.p);
    if (st) return st;
    if (mode != GALA_SOFTMAX_REF && mode != GALA_SOFTMAX_FIXED) return GALA_ERR_INVALID_ARG;
    if (F < 1 || F % heads != 0 || ldx < F || lddy < F) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0) return GALA_OK;
    if (!aL || (!aR && !wR) || !dY || !d_aL || (A->nnz > 0 && (!X || !alpha)))
        return GALA_ERR_INVALID_ARG;
    if (mode == GALA_SOFTMAX_FIXED && !d_logit && A->nnz > 0) return GALA_ERR_INVALID_ARG;
    if (!aR && mode != GALA_SOFTMAX_REF) return GALA_ERR_UNSUPPORTED;
    if (q && mode != GALA_SOFTMAX_REF) return GALA_ERR_INVALID_ARG;
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
    a.d.q = q;
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
                        alpha, nullptr, d_logit, d_aL, stream);
}

extern "C" int gala_gat_bwd_ex_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                   const float *wR, const float *bR, const float *X, int64_t ldx,
                                   const float *dY, int64_t lddy, int32_t F, int32_t heads,
                                   float slope, int32_t mode, const float *alpha, const float *q,
                                   float *d_logit, float *d_aL, void *stream) {
    if (!aR && !wR && A && A->n_rows > 0) return GALA_ERR_INVALID_ARG;
    return gat_bwd_impl(A, aL, aR, aR ? nullptr : wR, aR ? nullptr : bR, X, ldx, dY, lddy, F, heads,
                        slope, mode, alpha, q, d_logit, d_aL, stream);
}

extern "C" int gala_gat_bwd_attn_f32(const gala_csr_t *A, const float *aL, const float *wR,
                                     const float *bR, const float *X, int64_t ldx,
                                     const float *dY, int64_t lddy, int32_t F, float slope,
                                     const float *alpha, float *d_aL, void *stream) {
    if (!wR && A && A->n_rows > 0) return GALA_ERR_INVALID_ARG;
    return gat_bwd_impl(A, aL, nullptr, wR, bR, X, ldx, dY, lddy, F, 1, slope, GALA_SOFTMAX_REF,
                        alpha, nullptr, nullptr, d_aL, stream);
}

