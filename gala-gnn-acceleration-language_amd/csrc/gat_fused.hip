// gat_fused.hip -- the REF-mode GAT backward in one pass per row, with the attention
// recomputed instead of stored and the dX aggregation fused in.
//
// The reference's GAT backward (common.h:835-894, slot 2li+1 = the forward graph for the
// undirected graphs it runs) is dX = A_alpha dY (a weighted SpMM over the saved alpha)
// plus the edge chain edge_sddmm -> softmax bwd -> LeakyReLU bwd -> row sum.  Both walk
// the same rows over the same edges.  Here one row group does both: per edge it gathers
// X[col] (for d alpha = <dY[row], X[col]>) and dY[col] (for dX), and rebuilds
// alpha = fl(min(exp(LeakyReLU(aL[row] + aR[col])), 1e12) * q[row]) from the forward's
// per-row q = 1/(sum + 1e-12) -- the very product the forward would have stored -- so
// the forward writes no alpha (4 B per edge and head) and nothing reads it back.  aR is
// read, or recomputed per head from the gathered X row (wR, bR).
//
// Numerics: dX is accumulated sequentially in CSR order with fma(alpha, dY, acc), i.e.
// bit-identical to gala_spmm_f32 over the materialised alpha (hub rows: the same chunk
// partials and ordered fix-up).  d_aL's sums are taken per lane over the edges the lane
// owns and combined at the end of the row: equal to the reference within fp32 rounding.
#include "gat_common.h"

namespace gala {

struct FusedBwdState {
    float acc = 0.0f, s_msds = 0.0f, s_ma = 0.0f;
};

// Edges [e0, e1) of `row`: dX accumulators and the lane's share of the REF sums.  Edge k of
// a U-edge batch is owned by lane k mod UH of its head group: it loads / recomputes aR,
// forms alpha and the LeakyReLU factor, and counts the edge's sds; alpha is broadcast to
// the group for the dX accumulation.
// ST (row statistics, gala_gat_bwd_stats_f32): the d_aL sums come from the forward's rows,
// so an edge needs dY[col] and aR[col] only -- no X[col] gather, no per-edge dot.
template <int G, int VEC, int U, int HW, int CH, bool RC, bool ST>
__device__ __forceinline__ void gat_bwd_fused_range(const EdgeParams &p, const GatDev &d,
                                                    const GatLane<G, VEC, CH, RC> &gl_,
                                                    const float (&dy)[CH][VEC], int64_t e0,
                                                    int64_t e1, FusedBwdState &st,
                                                    float (&dxa)[CH][VEC]) {
    typedef typename GVec<VEC>::T V;
    constexpr int UH = (U < HW) ? U : HW;
    constexpr int NK = U / UH;
    const int H = gl_.H, hh = gl_.hh;
    const int lane = threadIdx.x & (kWave - 1);
    const int hl = lane & (HW - 1);
    const int kl = hl % UH;
    const bool owner = hl < UH;
    const int32_t n = (int32_t)(e1 - e0);
    int32_t win = 0;  // the row's next 64 column indices (load_batch_cols_win)
    for (int32_t j0 = 0; j0 < n; j0 += U) {
        int64_t c[U];
        V x[U][CH], yv[U][CH];
        load_batch_cols_win<G, U>(p, e0, n, j0, win, c);
        float ar[NK];
        // ST with the forward's p (d.alpha): alpha = fl(p * q) from the edge-ordered p,
        // no aR[col] gather
        const bool from_p = ST && d.alpha != nullptr;
        if (!RC) {
#pragma unroll
            for (int i = 0; i < NK; ++i) {
                const int32_t j = (j0 + kl + i * UH < n) ? j0 + kl + i * UH : n - 1;
                ar[i] = from_p ? d.alpha[(e0 + j) * H + hh] : d.aR[(int64_t)p.col[e0 + j] * H + hh];
            }
        }
#pragma unroll
        for (int k = 0; k < U; ++k)
#pragma unroll
            for (int ch = 0; ch < CH; ++ch) {
                if constexpr (!ST)
                    x[k][ch] = mask_pad<VEC>(gl_.ln.nv[ch], *reinterpret_cast<const V *>(d.X + c[k] * d.ldx + gl_.ln.off[ch]));
                // nontemporal: the gathered dY rows (2.5 GB at the Products shape, each read ~51
                // times at random) would otherwise evict the 78 MB aR table every edge also reads
                // (measured in one process: backward 26.1 -> 24.4 ms, tools/ab_gat.py)
                yv[k][ch] = mask_pad<VEC>(gl_.ln.nv[ch], __builtin_nontemporal_load(reinterpret_cast<const V *>(d.dY + c[k] * d.lddy + gl_.ln.off[ch])));
            }
        if constexpr (RC && !ST) {
            float all[U];
#pragma unroll
            for (int k = 0; k < U; ++k) all[k] = __fadd_rn(attn_dot<HW, VEC, CH>(gl_.w, x[k]), gl_.wb);
#pragma unroll
            for (int i = 0; i < NK; ++i) {
                float v = all[0];
#pragma unroll
                for (int k = 1; k < U; ++k) v = (kl + i * UH == k) ? all[k] : v;
                ar[i] = v;
            }
        }
        float a[NK];
        bool pos[NK];
#pragma unroll
        for (int i = 0; i < NK; ++i) {
            const float t = __fadd_rn(gl_.al, ar[i]);
            pos[i] = t > 0.0f;
            const float z = pos[i] ? t : __fmul_rn(t, d.slope);
            a[i] = __fmul_rn(from_p ? ar[i] : ref_exp(z), gl_.qr);
        }
        static_for<0, U>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            float dd = 0.0f;
            if constexpr (!ST) {
#pragma unroll
                for (int ch = 0; ch < CH; ++ch) {
                    const float *xv = reinterpret_cast<const float *>(&x[k][ch]);
#pragma unroll
                    for (int i = 0; i < VEC; ++i) dd = fmaf(dy[ch][i], xv[i], dd);
                }
                dd = group_sum<HW>(dd);
            }
            const float ak = group_bcast<HW, k % UH>(a[k / UH]);
            if (j0 + k >= n) return;
#pragma unroll
            for (int ch = 0; ch < CH; ++ch) {
                const float *yk = reinterpret_cast<const float *>(&yv[k][ch]);
#pragma unroll
                for (int i = 0; i < VEC; ++i) dxa[ch][i] = fmaf(ak, yk[i], dxa[ch][i]);
            }
            if (!ST && owner && kl == k % UH) {
                const int i = k / UH;
                const float sds = __fmul_rn(a[i], dd);
                st.acc += sds;
                st.s_msds += pos[i] ? sds : __fmul_rn(sds, d.slope);
                st.s_ma += pos[i] ? a[i] : __fmul_rn(a[i], d.slope);
            }
        });
    }
}

template <int G, int VEC, int CH>
__device__ __forceinline__ void store_dx(const GatDev &d, const Lanes<G, VEC, CH> &ln, float *base,
                                         const float (&dxa)[CH][VEC]) {
    typedef typename GVec<VEC>::T V;
#pragma unroll
    for (int ch = 0; ch < CH; ++ch) {
        if (!ln.valid[ch]) continue;
        V out;
        float *ov = reinterpret_cast<float *>(&out);
#pragma unroll
        for (int i = 0; i < VEC; ++i) ov[i] = dxa[ch][i];
        float *yp = base + ln.off[ch];
        if (ln.nv[ch] == VEC) {
            *reinterpret_cast<V *>(yp) = out;
        } else {
#pragma unroll
            for (int i = 0; i < VEC; ++i)
                if (ln.in(ch, i)) yp[i] = ov[i];
        }
    }
}

// The attention Linear's backward folded into the dX store: dX[r, f] += d_aL[r, head(f)] *
// w[f], with the roundings of gala_head_attn_bwd_f32 (a product, then a sum)
template <int G, int VEC, int CH>
__device__ __forceinline__ void add_attn_linear(const GatDev &d, const Lanes<G, VEC, CH> &ln, float dal,
                                                float (&dxa)[CH][VEC]) {
#pragma unroll
    for (int ch = 0; ch < CH; ++ch)
#pragma unroll
        for (int i = 0; i < VEC; ++i)
            if (ln.in(ch, i)) dxa[ch][i] = __fadd_rn(dxa[ch][i], __fmul_rn(dal, d.attn_w[ln.off[ch] + i]));
}

// d_aL of one row from the forward's row statistics: <dY, Y> and <dY, Ym> per head; every
// lane of the head returns the value its leader stores
template <int G, int VEC, int HW, int CH, bool RC>
__device__ __forceinline__ float stats_d_al(const EdgeParams &p, const GatDev &d, const GatLane<G, VEC, CH, RC> &gl_,
                                            int64_t row, const float (&dy)[CH][VEC]) {
    typedef typename GVec<VEC>::T V;
    float syy = 0.0f, sym = 0.0f;
#pragma unroll
    for (int ch = 0; ch < CH; ++ch) {
        const V y = mask_pad<VEC>(gl_.ln.nv[ch], *reinterpret_cast<const V *>(d.ys + row * d.ldy + gl_.ln.off[ch]));
        const V ym = mask_pad<VEC>(gl_.ln.nv[ch], *reinterpret_cast<const V *>(d.yms + row * d.ldym + gl_.ln.off[ch]));
        const float *yv = reinterpret_cast<const float *>(&y);
        const float *mv = reinterpret_cast<const float *>(&ym);
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
            syy = fmaf(dy[ch][i], yv[i], syy);
            sym = fmaf(dy[ch][i], mv[i], sym);
        }
    }
    const float eps = (float)p.seg.n * 1e-12f;
    const float acc = group_sum<HW>(syy) + eps;  // K7 on sds (common.h:793-794)
    const float s1 = group_sum<HW>(sym);
    if (!gl_.cv) return 0.0f;
    const int64_t o = row * gl_.H + gl_.hh;
    const float dal = (s1 - acc * d.smas[o]) + eps;   // common.h:662-667
    if (gl_.leader) d.d_aL[o] = dal;
    return dal;
}

template <int G, int VEC, int U, int HW, int CH, bool RC, bool ST>
__global__ __launch_bounds__(kBlock) void k_gat_bwd_fused(EdgeParams p, GatDev d, int32_t split_threshold) {
    GALA_ROW_PROLOGUE(G);
    if (!row_ok) return;
    const GatLane<G, VEC, CH, RC> gl_(p, d, gl, row);
    float dy[CH][VEC], dxa[CH][VEC];
    float dal = 0.0f;
    if constexpr (ST) {  // row-local: every row, hub rows included
        load_dy<G, VEC, CH, RC>(d, gl_, row, dy);
        dal = stats_d_al<G, VEC, HW, CH, RC>(p, d, gl_, row, dy);
    }
    if (split_threshold > 0 && p.rowptr[row + 1] - p.rowptr[row] > split_threshold)
        return;  // hub row: k_gat_bwd_fused_chunk / _fixup
    if constexpr (!ST) load_dy<G, VEC, CH, RC>(d, gl_, row, dy);
#pragma unroll
    for (int ch = 0; ch < CH; ++ch)
#pragma unroll
        for (int i = 0; i < VEC; ++i) dxa[ch][i] = 0.0f;
    FusedBwdState st;
    for (int s = 0; s < p.seg.n; ++s) {
        int64_t e0, e1;
        row_range(p, s, row, e0, e1);
        gat_bwd_fused_range<G, VEC, U, HW, CH, RC, ST>(p, d, gl_, dy, e0, e1, st, dxa);
    }
    if constexpr (ST)
        if (d.attn_w) add_attn_linear<G, VEC, CH>(d, gl_.ln, dal, dxa);
    store_dx<G, VEC, CH>(d, gl_.ln, d.dX + row * d.lddx, dxa);
    if constexpr (ST) return;
    const float eps = (float)p.seg.n * 1e-12f;
    const float acc = group_sum<HW>(st.acc) + eps;          // K7 on sds (common.h:793-794)
    const float s1 = group_sum<HW>(st.s_msds), s2 = group_sum<HW>(st.s_ma);
    if (gl_.leader) d.d_aL[row * gl_.H + gl_.hh] = (s1 - acc * s2) + eps;  // common.h:662-667
}

// hub rows: chunk partials -> ws[c] = {dX[F], acc[H], s_msds[H], s_ma[H]}
template <int G, int VEC, int U, int HW, int CH, bool RC, bool ST>
__global__ __launch_bounds__(kBlock) void k_gat_bwd_fused_chunk(EdgeParams p, GatDev d, HubSplit sp) {
    GALA_CHUNK_PROLOGUE(G);
    const GatLane<G, VEC, CH, RC> gl_(p, d, gl, row);
    float dy[CH][VEC], dxa[CH][VEC];
    if constexpr (!ST) load_dy<G, VEC, CH, RC>(d, gl_, row, dy);
#pragma unroll
    for (int ch = 0; ch < CH; ++ch)
#pragma unroll
        for (int i = 0; i < VEC; ++i) dxa[ch][i] = 0.0f;
    FusedBwdState st;
    gat_bwd_fused_range<G, VEC, U, HW, CH, RC, ST>(p, d, gl_, dy, e0, e1, st, dxa);
    float *w = sp.ws + c * sp.ws_cols;
    store_dx<G, VEC, CH>(d, gl_.ln, w, dxa);
    if constexpr (ST) return;  // ws[c] = {dX[F]}
    const float acc = group_sum<HW>(st.acc);
    const float s1 = group_sum<HW>(st.s_msds), s2 = group_sum<HW>(st.s_ma);
    if (gl_.leader) {
        const int F = d.F, H = gl_.H, hh = gl_.hh;
        w[F + hh] = acc;
        w[F + H + hh] = s1;
        w[F + 2 * H + hh] = s2;
    }
}

// hub rows: the chunk partials of a row summed in chunk order (dX: as k_spmm_fixup)
template <int G, int VEC, int CH, bool RC, bool ST>
__global__ __launch_bounds__(kBlock) void k_gat_bwd_fused_fixup(EdgeParams p, GatDev d, HubSplit sp) {
    const int lane = threadIdx.x & (kWave - 1);
    const int gl = lane & (G - 1);
    const int64_t ri = ((int64_t)blockIdx.x * (kBlock / kWave) + threadIdx.x / kWave) * (kWave / G) + lane / G;
    if (ri >= sp.n_rows_split) return;
    const int64_t row = sp.rows[ri];
    const GatLane<G, VEC, CH, RC> gl_(p, d, gl, row);
    const int F = d.F, H = gl_.H, hh = gl_.hh;
    float dxa[CH][VEC];
#pragma unroll
    for (int ch = 0; ch < CH; ++ch)
#pragma unroll
        for (int i = 0; i < VEC; ++i) dxa[ch][i] = 0.0f;
    float acc = 0.0f, s1 = 0.0f, s2 = 0.0f;
    for (int64_t cc = sp.row_chunk0[ri]; cc < sp.row_chunk0[ri + 1]; ++cc) {
        const float *w = sp.ws + cc * sp.ws_cols;
#pragma unroll
        for (int ch = 0; ch < CH; ++ch)
#pragma unroll
            for (int i = 0; i < VEC; ++i)
                dxa[ch][i] = __fadd_rn(dxa[ch][i], gl_.ln.in(ch, i) ? w[gl_.ln.off[ch] + i] : 0.0f);
        if constexpr (!ST) {
            acc = __fadd_rn(acc, w[F + hh]);
            s1 = __fadd_rn(s1, w[F + H + hh]);
            s2 = __fadd_rn(s2, w[F + 2 * H + hh]);
        }
    }
    if constexpr (ST)  // the row's d_aL was stored by k_gat_bwd_fused
        if (d.attn_w && gl_.cv) add_attn_linear<G, VEC, CH>(d, gl_.ln, d.d_aL[row * H + hh], dxa);
    store_dx<G, VEC, CH>(d, gl_.ln, d.dX + row * d.lddx, dxa);
    if (!ST && gl_.leader) {
        acc = __fadd_rn(acc, 1e-12f);
        d.d_aL[row * H + hh] = (s1 - acc * s2) + 1e-12f;
    }
}

}  // namespace gala

using namespace gala;

namespace {

struct FusedArgs {
    EdgeParams p;
    GatDev d;
    HubSplit sp;
    bool split;
    hipStream_t hs;
};

template <int G, int VEC, int HW, int CH, bool RC, bool ST>
void launch_fused_st(const FusedArgs &a) {
    constexpr int U = 8;
    hipLaunchKernelGGL((k_gat_bwd_fused<G, VEC, U, HW, CH, RC, ST>), dim3(blocks_for(a.p.n_rows, G)), dim3(kBlock),
                       0, a.hs, a.p, a.d, a.split ? a.sp.threshold : 0);
    if (!a.split) return;
    hipLaunchKernelGGL((k_gat_bwd_fused_chunk<G, VEC, U, HW, CH, RC, ST>), dim3(blocks_for_groups(a.sp.n_chunks, G)),
                       dim3(kBlock), 0, a.hs, a.p, a.d, a.sp);
    hipLaunchKernelGGL((k_gat_bwd_fused_fixup<G, VEC, CH, RC, ST>), dim3(blocks_for_groups(a.sp.n_rows_split, G)),
                       dim3(kBlock), 0, a.hs, a.p, a.d, a.sp);
}

// RC: aR recomputed from X (never with the statistics, which read aR); !RC: the
// statistics variant when the forward's rows are given (a.d.ys)
template <int G, int VEC, int HW, int CH, bool RC>
void launch_fused(const FusedArgs &a) {
    if constexpr (RC) launch_fused_st<G, VEC, HW, CH, true, false>(a);
    else if (a.d.ys) launch_fused_st<G, VEC, HW, CH, false, true>(a);
    else launch_fused_st<G, VEC, HW, CH, false, false>(a);
}

template <int G, int VEC, bool RC>
int fused_g(const FusedArgs &a, int heads, int hw) {
    if (heads == 1) {
        launch_fused<G, VEC, G, 1, RC>(a);
        return GALA_OK;
    }
    if constexpr (G >= 2) {
        switch (hw) {
            case 1: launch_fused<G, VEC, 1, 1, RC>(a); return GALA_OK;
            case 2: if constexpr (G > 2) { launch_fused<G, VEC, 2, 1, RC>(a); return GALA_OK; } break;
            case 4: if constexpr (G > 4) { launch_fused<G, VEC, 4, 1, RC>(a); return GALA_OK; } break;
            case 8: if constexpr (G > 8) { launch_fused<G, VEC, 8, 1, RC>(a); return GALA_OK; } break;
            case 16: if constexpr (G > 16) { launch_fused<G, VEC, 16, 1, RC>(a); return GALA_OK; } break;
            case 32: if constexpr (G > 32) { launch_fused<G, VEC, 32, 1, RC>(a); return GALA_OK; } break;
            default: break;
        }
    }
    return GALA_ERR_UNSUPPORTED;
}

template <int VEC, bool RC>
int fused_vec(const FusedArgs &a, int L, int ch, int heads, int hw) {
    if (ch == 2) launch_fused<16, VEC, 16, 2, RC>(a);
    else if (ch == 3) launch_fused<16, VEC, 16, 3, RC>(a);
    else if (ch == 4) launch_fused<16, VEC, 16, 4, RC>(a);
    else if (L <= 1) launch_fused<1, VEC, 1, 1, RC>(a);
    else if (L <= 2) return fused_g<2, VEC, RC>(a, heads, hw);
    else if (L <= 4) return fused_g<4, VEC, RC>(a, heads, hw);
    else if (L <= 8) return fused_g<8, VEC, RC>(a, heads, hw);
    else if (L <= 16) return fused_g<16, VEC, RC>(a, heads, hw);
    else if (L <= 32) return fused_g<32, VEC, RC>(a, heads, hw);
    else if (L <= 64) return fused_g<64, VEC, RC>(a, heads, hw);
    else return GALA_ERR_UNSUPPORTED;
    return GALA_OK;
}

}  // namespace

static int fused_dispatch(FusedArgs &a, int F, int heads, int vec, bool rc) {
    const int D = F / heads;
    const int L = (F + vec - 1) / vec;
    const int ch = narrow_chunks(heads, vec, L);
    const int hw = (D % vec == 0) ? D / vec : 0;
    if (heads > 1 && (hw == 0 || (hw & (hw - 1)))) return GALA_ERR_UNSUPPORTED;
    int r;
    if (vec == 4) r = rc ? fused_vec<4, true>(a, L, ch, heads, hw) : fused_vec<4, false>(a, L, ch, heads, hw);
    else if (vec == 2) r = rc ? fused_vec<2, true>(a, L, ch, heads, hw) : fused_vec<2, false>(a, L, ch, heads, hw);
    else r = rc ? fused_vec<1, true>(a, L, ch, heads, hw) : fused_vec<1, false>(a, L, ch, heads, hw);
    if (r) return r;
    return launch_status();
}

static int bwd_stats_impl(const gala_csr_t *A, const float *aL, const float *aR, const float *pe,
                          const float *dY, int64_t lddy, const float *dY_rows, int32_t F, int32_t heads,
                          float slope, const float *q, const float *Y, int64_t ldy, const float *Ym,
                          int64_t ldym, const float *sma, float *dX, int64_t lddx, float *d_aL, void *stream,
                          const float *wR = nullptr) {
    FusedArgs a{};
    int st = edge_setup(A, heads, &a.p);
    if (st) return st;
    if (F < 1 || F % heads != 0 || lddy < F || ldy < F || ldym < F || lddx < F) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0) return GALA_OK;
    if (!aL || (!aR && !pe) || !q || !dY || !Y || !Ym || !sma || !dX || !d_aL) return GALA_ERR_INVALID_ARG;
    // dY[col] and dY[row] are one array for a square pattern; a gathered table (a row
    // partition's halo) passes the rows' own dY apart
    if (!dY_rows && A->n_cols > A->n_rows && A->nnz > 0) return GALA_ERR_INVALID_ARG;
    if (dY_rows && ((uintptr_t)dY_rows % 16) != ((uintptr_t)dY % 16)) return GALA_ERR_INVALID_ARG;
    const int D = F / heads;
    auto ok = [&](int v) {
        const bool fits = D % v == 0 || (heads == 1 && lddy >= pad_to(F, v) && ldy >= pad_to(F, v) &&
                                         ldym >= pad_to(F, v) && lddx >= pad_to(F, v));
        return fits && lddy % v == 0 && ldy % v == 0 && ldym % v == 0 && lddx % v == 0 &&
               ((uintptr_t)dY % (4 * v)) == 0 && ((uintptr_t)Y % (4 * v)) == 0 &&
               ((uintptr_t)Ym % (4 * v)) == 0 && ((uintptr_t)dX % (4 * v)) == 0;
    };
    int vec = 4;
    while (vec > 1 && !ok(vec)) vec >>= 1;
    a.d.aL = aL, a.d.aR = aR, a.d.F = F, a.d.slope = slope;
    a.d.dY = dY, a.d.lddy = lddy, a.d.q = q, a.d.dX = dX, a.d.lddx = lddx, a.d.d_aL = d_aL;
    a.d.ys = Y, a.d.ldy = ldy, a.d.yms = Ym, a.d.ldym = ldym, a.d.smas = sma, a.d.alpha = pe;
    a.d.dy_rows = dY_rows;
    a.d.attn_w = wR;
    a.hs = (hipStream_t)stream;
    a.split = hub_split(A, pad_to(F, 4), &a.sp);  // hub rows: dX[F] chunk partials
    return fused_dispatch(a, F, heads, vec, false);
}

extern "C" int gala_gat_bwd_stats_f32(const gala_csr_t *A, const float *aL, const float *aR, const float *pe,
                                      const float *dY, int64_t lddy, int32_t F, int32_t heads, float slope, const float *q,
                                      const float *Y, int64_t ldy, const float *Ym, int64_t ldym,
                                      const float *sma, float *dX, int64_t lddx, float *d_aL, void *stream) {
    return bwd_stats_impl(A, aL, aR, pe, dY, lddy, nullptr, F, heads, slope, q, Y, ldy, Ym, ldym, sma, dX, lddx,
                          d_aL, stream);
}

extern "C" int gala_gat_bwd_stats_ex_f32(const gala_csr_t *A, const float *aL, const float *aR, const float *pe,
                                         const float *dY, int64_t lddy, const float *dY_rows, int32_t F,
                                         int32_t heads, float slope, const float *q, const float *Y, int64_t ldy,
                                         const float *Ym, int64_t ldym, const float *sma, float *dX, int64_t lddx,
                                         float *d_aL, void *stream) {
    return bwd_stats_impl(A, aL, aR, pe, dY, lddy, dY_rows, F, heads, slope, q, Y, ldy, Ym, ldym, sma, dX, lddx,
                          d_aL, stream);
}

// The same with the source logit's per-head Linear (aR = X wR + bR) folded in: dX also
// takes d_aR * wR (REF: d_aR = d_aL), bit-identical to gala_head_attn_bwd_f32 accumulating
// into the statistics backward's dX.
extern "C" int gala_gat_bwd_stats_linear_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                             const float *pe, const float *dY, int64_t lddy, const float *dY_rows,
                                             int32_t F, int32_t heads, float slope, const float *q, const float *Y,
                                             int64_t ldy, const float *Ym, int64_t ldym, const float *sma,
                                             const float *wR, float *dX, int64_t lddx, float *d_aL, void *stream) {
    if (!wR && A && A->n_rows > 0) return GALA_ERR_INVALID_ARG;
    return bwd_stats_impl(A, aL, aR, pe, dY, lddy, dY_rows, F, heads, slope, q, Y, ldy, Ym, ldym, sma, dX, lddx,
                          d_aL, stream, wR);
}

extern "C" int gala_gat_bwd_fused_f32(const gala_csr_t *A, const float *aL, const float *aR,
                                      const float *wR, const float *bR, const float *X,
                                      int64_t ldx, const float *dY, int64_t lddy, int32_t F,
                                      int32_t heads, float slope, const float *q, float *dX,
                                      int64_t lddx, float *d_aL, void *stream) {
    FusedArgs a{};
    int st = edge_setup(A, heads, &a.p);
    if (st) return st;
    if (F < 1 || F % heads != 0 || ldx < F || lddy < F || lddx < F) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0) return GALA_OK;
    if (!aL || (!aR && !wR) || !q || !dY || !dX || !d_aL || (A->nnz > 0 && !X)) return GALA_ERR_INVALID_ARG;
    if (A->n_cols > A->n_rows && A->nnz > 0) return GALA_ERR_INVALID_ARG;  // dY[col]: a square pattern
    const int D = F / heads;
    int vec = 4;
    auto ok = [&](int v) {
        const bool fits = D % v == 0 || (heads == 1 && ldx >= pad_to(F, v) && lddy >= pad_to(F, v) &&
                                         lddx >= pad_to(F, v));
        return fits && ldx % v == 0 && lddy % v == 0 && lddx % v == 0 && ((uintptr_t)X % (4 * v)) == 0 &&
               ((uintptr_t)dY % (4 * v)) == 0 && ((uintptr_t)dX % (4 * v)) == 0;
    };
    while (vec > 1 && !ok(vec)) vec >>= 1;
    const int L = (F + vec - 1) / vec;
    const int ch = narrow_chunks(heads, vec, L);
    int G = 16;
    if (ch == 1) {
        G = 1;
        while (G < L) G <<= 1;
    }
    const int hw = (D % vec == 0) ? D / vec : 0;
    if (heads > 1 && (hw == 0 || (hw & (hw - 1)))) return GALA_ERR_UNSUPPORTED;
    a.d.aL = aL, a.d.aR = aR, a.d.wR = aR ? nullptr : wR, a.d.bR = aR ? nullptr : bR;
    a.d.X = X, a.d.ldx = ldx, a.d.F = F, a.d.slope = slope;
    a.d.dY = dY, a.d.lddy = lddy, a.d.q = q, a.d.dX = dX, a.d.lddx = lddx, a.d.d_aL = d_aL;
    a.hs = (hipStream_t)stream;
    a.split = hub_split(A, pad_to(F, 4) + 3 * (int64_t)heads, &a.sp);
    const bool rc = aR == nullptr;
    int r;
    if (vec == 4) r = rc ? fused_vec<4, true>(a, L, ch, heads, hw) : fused_vec<4, false>(a, L, ch, heads, hw);
    else if (vec == 2) r = rc ? fused_vec<2, true>(a, L, ch, heads, hw) : fused_vec<2, false>(a, L, ch, heads, hw);
    else r = rc ? fused_vec<1, true>(a, L, ch, heads, hw) : fused_vec<1, false>(a, L, ch, heads, hw);
    if (r) return r;
    return launch_status();
}
