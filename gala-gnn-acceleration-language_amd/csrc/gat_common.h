// gat_common.h -- shared by the fused GAT kernels (gat.hip: forward and the alpha-based
// backward; gat_fused.hip: the REF backward with recomputed attention and fused dX): the
// operand block, the per-lane view of a row, the attention recompute.
#pragma once

#include <type_traits>

#include "edge_common.h"

namespace gala {

// RC (one head): the source logit aR[col] = <X[col,:], wR> + bR is recomputed from the X
// row the aggregation gathers anyway (the DSL's attnR = dsl.nn.ffn(res, out=1) of the
// aggregated `res`, tests/GALA-DSL/gat/*), instead of a separate random aR[col] read.
// The columns of edges j0 .. j0+U-1 of a row (clamped to the row's last edge).  With one
// row per wave (G = 64) they are wave-uniform: one coalesced load of the U columns, spread
// to scalar registers with v_readlane, so the gathered rows' addresses are formed on the
// scalar unit (about 6 VALU instructions per edge and lane otherwise).
template <int G, int U>
__device__ __forceinline__ void load_batch_cols(const EdgeParams &p, int64_t e0, int32_t n, int32_t j0,
                                                int64_t (&c)[U]) {
    if constexpr (G == 64) {
        const int kk = threadIdx.x & (U - 1);
        const int32_t cu = p.col[e0 + ((j0 + kk < n) ? j0 + kk : n - 1)];
#pragma unroll
        for (int k = 0; k < U; ++k) c[k] = __builtin_amdgcn_readlane(cu, k);
    } else {
#pragma unroll
        for (int k = 0; k < U; ++k) c[k] = p.col[e0 + ((j0 + k < n) ? j0 + k : n - 1)];
    }
}

// The same columns from a window of the row's next 64 column indices held one per lane
// (G = 64, U | 64): one coalesced load per 64 edges instead of one per U-edge batch, so a
// batch's gathers wait on one memory round trip (the X rows) rather than two (the column
// indices, then the rows).  `win` carries the window between batches; j0 steps by U from 0.
template <int G, int U>
__device__ __forceinline__ void load_batch_cols_win(const EdgeParams &p, int64_t e0, int32_t n, int32_t j0,
                                                    int32_t &win, int64_t (&c)[U]) {
    if constexpr (G == 64 && (64 % U) == 0) {
        const int lane = threadIdx.x & 63;
        const int b = j0 & 63;
        if (b == 0) win = p.col[e0 + ((j0 + lane < n) ? j0 + lane : n - 1)];
#pragma unroll
        for (int k = 0; k < U; ++k) c[k] = __builtin_amdgcn_readlane(win, b + k);
    } else {
        load_batch_cols<G, U>(p, e0, n, j0, c);
    }
}

// Broadcast of lane SRC of each aligned group of HW lanes to the group, SRC a compile-time
// constant.  HW <= 16: DPP moves inside the 16-lane row (quad_perm picks lane SRC % 4 of each
// quad; a row shift by 4, then 8, carries it to the group's other quads), VALU only; HW = 32:
// ds_swizzle in bitmask mode (no address VGPR, unlike ds_bpermute); a whole wave: v_readlane.
template <int HW, int SRC>
__device__ __forceinline__ float group_bcast(float v) {
    if constexpr (HW == 1) {
        return v;
    } else if constexpr (HW == 2) {
        constexpr int c = SRC | (SRC << 2) | ((2 + SRC) << 4) | ((2 + SRC) << 6);
        return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), c, 0xF, 0xF, true));
    } else if constexpr (HW <= 16) {
        constexpr int s = SRC & 3;
        int t = __builtin_amdgcn_mov_dpp(__float_as_int(v), s | (s << 2) | (s << 4) | (s << 6), 0xF, 0xF, true);
        if constexpr (HW >= 8) {   // quad SRC / 4 of each 8-lane group to the other quad
            constexpr int q = (SRC >> 2) & 1;
            const int u = __builtin_amdgcn_mov_dpp(t, q ? 0x104 : 0x114, 0xF, 0xF, true);
            t = (((threadIdx.x >> 2) & 1) == q) ? t : u;
        }
        if constexpr (HW == 16) {  // 8-lane half SRC / 8 to the other half
            constexpr int h = (SRC >> 3) & 1;
            const int u = __builtin_amdgcn_mov_dpp(t, h ? 0x108 : 0x118, 0xF, 0xF, true);
            t = (((threadIdx.x >> 3) & 1) == h) ? t : u;
        }
        return __int_as_float(t);
    } else if constexpr (HW <= 32) {
        constexpr int pattern = (0x1F & ~(HW - 1)) | (SRC << 5);  // lane' = (lane & and) | or
        return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), pattern));
    } else {
        return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), SRC));
    }
}

// f(std::integral_constant<int, K>) for K = B .. E-1 (compile-time loop index)
template <int B, int E, typename Fn>
__device__ __forceinline__ void static_for(Fn &&f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// With several heads the dot runs over the head's HW lanes (its slice of X and wR): the
// standard multi-head GAT source logit <X[col, hD:(h+1)D], wR[hD:(h+1)D]> + bR[h].
template <int HW, int VEC, int CH>
__device__ __forceinline__ float attn_dot(const float (&w)[CH][VEC],
                                          const typename GVec<VEC>::T (&x)[CH]) {
    float d = 0.0f;
#pragma unroll
    for (int ch = 0; ch < CH; ++ch) {
        const float *xv = reinterpret_cast<const float *>(&x[ch]);
#pragma unroll
        for (int i = 0; i < VEC; ++i) d = fmaf(w[ch][i], xv[i], d);
    }
    return group_sum<HW>(d);
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
    const float *dY, *alpha;         // backward (alpha: p when q != nullptr)
    const float *q;                  // backward, nullable: alpha = p * q[row, h] (REF, factored)
    float *Y, *alpha_out;            // forward (alpha_out: p when q_out != nullptr)
    float *q_out;                    // forward, nullable: factored attention output (REF)
    float *d_logit, *d_aL;           // backward
    float *dX;                       // fused REF backward: dX = A_alpha dY (forward pattern)
    int64_t ldx, ldy, lddy, lddx;
    int32_t F;
    float slope;
    int32_t partial;                 // forward, GALA_GAT_PARTIAL: unnormalised Y, raw sums in q_out
    // REF row statistics (gala_gat_{fwd,bwd}_stats_f32): Ym = sum m*alpha*X, sma = sum m*alpha
    float *ym_out, *sma_out, *ar_out;  // forward (ar_out: the rows' recomputed aR, nullable)
    const int32_t *self_col;           // forward with ar_out, nullable: the column of each row's own
                                       // vertex (-1: not held); NULL = the row itself (square)
    const float *ys, *yms, *smas;      // backward: Y (ld ldy), Ym (ld ldym), sma
    const float *dy_rows;              // backward, nullable: the rows' own dY (row r at dy_rows + r*lddy)
                                       // when dY is a gathered table whose row r is not column r
    int64_t ldym;
    // forward continuation (gala_gat_fwd_continue_f32, REF): each row's state starts from the
    // unnormalised partials {sum p X, sum p[, sum m p X, sum m p]} of an earlier pass over
    // other columns; they may alias Y, q_out, Ym and sma (each lane reads its own elements
    // before it writes them)
    const float *init_acc, *init_sum, *init_accm, *init_sma;
    int64_t ld_init, ld_initm;
    // statistics backward, nullable: the source logit's per-head Linear weights [F] (aR = X wR
    // + bR); dX[r, f] += d_aL[r, head(f)] * attn_w[f] at the store (REF: d_aR = d_aL)
    const float *attn_w;
};

// Internal forward MODE: REF softmax that also accumulates the row statistics.
constexpr int kRefStats = 2;
__host__ __device__ constexpr bool ref_mode(int mode) { return mode != GALA_SOFTMAX_FIXED; }


// The lane's share of one row (or one chunk of a hub row) for the GAT kernels.
template <int G, int VEC, int CH, bool RC>
struct GatLane {
    Lanes<G, VEC, CH> ln;
    int H, D, hh;
    bool cv, leader;
    float al, wb, qr;
    float w[CH][VEC];
    __device__ __forceinline__ GatLane(const EdgeParams &p, const GatDev &d, int gl, int64_t row)
        : ln(gl, d.F) {
        H = p.heads;  // CH > 1 and RC only with H == 1
        D = d.F / H;
        cv = ln.valid[0];
        hh = (int)(ln.off[0] / D);
        leader = cv && (ln.off[0] % D) == 0;
        al = d.aL[row * H + hh];
        qr = d.q ? d.q[row * H + hh] : 1.0f;
        wb = 0.0f;
        if (RC) {
            load_attn<G, VEC, CH>(ln, d.wR, w);
            wb = d.bR ? d.bR[hh] : 0.0f;
        }
    }
};

template <int G, int VEC, int CH, bool RC>
__device__ __forceinline__ void load_dy(const GatDev &d, const GatLane<G, VEC, CH, RC> &gl_, int64_t row,
                                        float (&dy)[CH][VEC]) {
    typedef typename GVec<VEC>::T V;
    const float *base = d.dy_rows ? d.dy_rows : d.dY;
#pragma unroll
    for (int ch = 0; ch < CH; ++ch) {
        const V t = *reinterpret_cast<const V *>(base + row * d.lddy + gl_.ln.off[ch]);
#pragma unroll
        for (int i = 0; i < VEC; ++i) dy[ch][i] = gl_.ln.in(ch, i) ? reinterpret_cast<const float *>(&t)[i] : 0.0f;
    }
}


}  // namespace gala
