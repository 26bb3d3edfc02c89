// gat_input.hip -- config 3's multi-head GAT layer in input space (round 6).
//
// The layer (tests/GALA-DSL/gat/*, galac gat_heads(H)) is
//     v1 = Xin W^T + b                 FFN_OP, Xin [N, fin] -> H heads of D
//     aL = head_attn(v1, wL, bL)       attnL = dsl.nn.ffn(res, out=1) per head
//     aR = head_attn(v1, wR, bR)       attnR, recomputed from the aggregated rows
//     Y  = REF GAT(aL, aR, v1)         K5 -> LeakyReLU -> softmax -> weighted aggregation
// and the reference gathers v1[col] -- H*D floats, 1 KB per edge at config 3 -- for every
// edge of the forward, and dY[col] for every edge of the backward.  Per head the aggregation
// is linear in v1, so with alpha = p * q (p per edge, q per row):
//     Y_h[r]  = q_h[r] * (sum_e p_e,h Xin_ext[c_e]) W_ext,h^T       (Xin_ext = [Xin, 1],
//     Ym_h[r] = q_h[r] * (sum_e m_e p_e,h Xin_ext[c_e]) W_ext,h^T    W_ext = [W, b])
//     aL / aR = Xin uL/uR^T + betaL/R, uL_h = W_h^T wL_h, betaL_h = b_h . wL_h + bL_h
// so the forward gathers the 400-B input row instead (fin = 100), accumulates the per-head
// aggregates of the input rows on the matrix cores (v_mfma_f32_16x16x4_f32, exact f32: edges
// are the k dimension) and projects each row's aggregates with W_ext,h in the epilogue -- one
// workgroup phase projects eight rows per head, so W's fragments stay in registers.  The
// REF backward (common.h:835-894: dX[r] = sum_{e in row r} alpha_e dY[c_e] with the forward
// alpha) only feeds the FFN's weight gradient, which regroups by column:
//     sum_r dX[r]^T Xin_ext[r] = sum_c dY[c]^T T[c],   T_h[c] = sum_{e: c_e = c} alpha_e,h Xin_ext[r_e]
// over the transposed pattern: the backward gathers the 512-B extended input row (with aL and
// q riding in its padding) instead of 1 KB of dY plus an aR line, and never forms dX.
//
// Extended rows (kInLd = 128 floats, written by k_gat_in_prep every forward).  The
// aggregation kernels read a row as two float4 per lane over 16 lanes: lane n holds slots
// 4n..4n+3 and 64+4n..64+4n+3.
//     slots 0..63            features 0..63
//     64+4n+{0,1,2}, n < 12  features 64+3n .. 64+3n+2 (features 64..99)
//     112 (lane 12 .x)       1.0: the ones column (sum p, and the bias through W_ext)
//     64+4h+3, h < 8         aR[h]  (lane h's .w: the forward's source logit, no extra line)
//     96+4h+3, h < 8         aL[h]  (lane 8+h's .w: read by the transposed backward)
//     116+4(h/3)+h%3         q[h]   (lanes 13..15 .xyz: written by the forward's projection)
// MFMA feature tile t (k order of the aggregation): t < 4 is the first float4's component t
// (feature 4n + t), t = 4..6 the second float4's component t - 4.
//
// Numerics (north_star: fp32 within 1e-4 of the reference): the per-edge terms are the
// reference's -- t = fl(aL + aR), LeakyReLU, clamp(exp(t), 1e12), alpha = fl(p * q) in the
// backward -- and every sum is an f32 fmaf chain, regrouped (edge order inside an MFMA k-step,
// the input-space association); the layer is checked against the oracle's pass-by-pass REF
// layer at the Products shape (tests/test_gpu_gat_input.py).
#include <cstdlib>

#include "edge_common.h"

namespace gala {
namespace {

typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int kInLd = 128;
constexpr int kInMaxFin = 100;
constexpr int kInMaxHeads = 8;
constexpr int kInWaves = 8;              // waves per workgroup = rows (columns) per phase
constexpr int kInBlock = kInWaves * kWave;
constexpr int kInTiles = 7;              // feature tiles of 16
constexpr int kInGrid = 512;             // persistent workgroups (2 per CU)
constexpr int kOnesSlot = 112;

__host__ __device__ constexpr int ext_slot(int f) { return f < 64 ? f : 64 + 4 * ((f - 64) / 3) + (f - 64) % 3; }
__host__ __device__ constexpr int aR_slot(int h) { return 67 + 4 * h; }
__host__ __device__ constexpr int aL_slot(int h) { return 99 + 4 * h; }
__host__ __device__ constexpr int q_slot(int h) { return 116 + 4 * (h / 3) + h % 3; }

// input feature of row m of feature tile t: >= 0 a feature, -2 the ones column, -1 padding
__device__ __forceinline__ int tile_feature(int t, int m, int fin) {
    int f;
    if (t < 4) f = 4 * m + t;
    else if (m < 12) f = 64 + 3 * m + (t - 4);
    else return (m == 12 && t == 4) ? -2 : -1;
    return f < fin ? f : -1;
}

__device__ __forceinline__ f4v mfma4(float a, float b, f4v c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// lane i <- lane i +- 8 inside its 16-lane row (row_ror:8)
__device__ __forceinline__ float ror8(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xF, 0xF, true));
}

struct InPrepParams {
    const float *X;
    int64_t n, ldx;
    int32_t fin, H;
    const float *u;   // [2H][fin]: uL rows, then uR rows
    const float *c;   // [2H]: betaL, betaR
    float *xext;
};

// 16 lanes per row, each owning the two float4 slots the aggregation kernels read (lane n:
// features 4n..4n+3, and 64+3n..64+3n+2 for n < 12): the row's 2H logits are per-lane partial
// dots (u held in registers for the lane's seven features, the grid persistent) summed by a
// 16-lane butterfly, then every lane stores its two float4 (the row's 512 B, coalesced).
__global__ __launch_bounds__(kBlock) void k_gat_in_prep(InPrepParams p) {
    const int lane = threadIdx.x & 63, n = lane & 15;
    const int64_t g0 = (int64_t)blockIdx.x * (kBlock / 16) + threadIdx.x / 16, gstep = (int64_t)gridDim.x * (kBlock / 16);
    const int K = 2 * p.H;
    float ua[2 * kInMaxHeads][4], ub[2 * kInMaxHeads][3];
#pragma unroll
    for (int k = 0; k < 2 * kInMaxHeads; ++k) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int f = 4 * n + i;
            ua[k][i] = (k < K && f < p.fin) ? p.u[k * p.fin + f] : 0.0f;
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const int f = 64 + 3 * n + i;
            ub[k][i] = (k < K && n < 12 && f < p.fin) ? p.u[k * p.fin + f] : 0.0f;
        }
    }
    const float cl = n >= 8 && n - 8 < p.H ? p.c[n - 8] : 0.0f;     // lane 8+h: aL[h]'s constant
    const float cr = n < 8 && n < p.H ? p.c[p.H + n] : 0.0f;       // lane h: aR[h]'s
    for (int64_t r = g0; r < p.n; r += gstep) {
        const float *x = p.X + r * p.ldx;
        float xa[4], xb[3];
#pragma unroll
        for (int i = 0; i < 4; ++i) xa[i] = 4 * n + i < p.fin ? x[4 * n + i] : 0.0f;
#pragma unroll
        for (int i = 0; i < 3; ++i) xb[i] = (n < 12 && 64 + 3 * n + i < p.fin) ? x[64 + 3 * n + i] : 0.0f;
        float lg[2 * kInMaxHeads];
#pragma unroll
        for (int k = 0; k < 2 * kInMaxHeads; ++k) {
            float d = 0.0f;
#pragma unroll
            for (int i = 0; i < 4; ++i) d = fmaf(xa[i], ua[k][i], d);
#pragma unroll
            for (int i = 0; i < 3; ++i) d = fmaf(xb[i], ub[k][i], d);
            lg[k] = group_sum<16>(d);
        }
        // lane h < 8: aR[h] = lg[H + h] + cR; lane 8 + h: aL[h] = lg[h] + cL
        float w = 0.0f;
#pragma unroll
        for (int k = 0; k < 2 * kInMaxHeads; ++k) {
            if (n < 8 && k == p.H + n) w = lg[k];
            if (n >= 8 && k == n - 8) w = lg[k];
        }
        w = (n < 8 ? (n < p.H) : (n - 8 < p.H)) ? __fadd_rn(w, n < 8 ? cr : cl) : 0.0f;
        f4v A = f4v{xa[0], xa[1], xa[2], xa[3]};
        f4v B = n < 12 ? f4v{xb[0], xb[1], xb[2], w} : f4v{n == 12 ? 1.0f : 0.0f, 0.0f, 0.0f, w};
        float *o = p.xext + r * kInLd;
        *reinterpret_cast<f4v *>(o + 4 * n) = A;
        *reinterpret_cast<f4v *>(o + 64 + 4 * n) = B;
    }
}

struct InFwdParams {
    const int32_t *rowptr, *col, *order;
    int64_t n_rows;
    float *xext;
    const float *W, *b;
    int64_t ldw;
    int32_t fin, H, D;
    float slope;
    float *Y, *Ym, *q, *sma;
    int64_t ldy;
    int32_t relu;   // GALA_GAT_IN_RELU: Y = relu(the aggregation) (the layer's NON_LNR_OP_RELU)
    float *T;       // T mode: the backward's per-column aggregates (see k_gat_in_fwd), else null
};

// the gathered extended row of edge (4s + kq) of a 16-edge batch: column from the row's
// 64-index window (lane i holds col[e0 + j0w + i])
__device__ __forceinline__ int64_t batch_col(int32_t win, int j0, int s, int kq) {
    const int src = (j0 & 63) + 4 * s + kq;
    return (int64_t)__builtin_amdgcn_ds_bpermute(src * 4, win);
}

// the 16-edge batch j0 of a row: lane (16 kq + n) requests slots 4n.. and 64+4n.. of the
// extended rows of edges j0 + 4s + kq (s = 0..3)
__device__ __forceinline__ void load_batch(const float *xext, int32_t win, int32_t j0, int kq, int n16,
                                           f4v (&xa)[4], f4v (&xb)[4]) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int64_t c = batch_col(win, j0, s, kq);
        xa[s] = *reinterpret_cast<const f4v *>(xext + c * kInLd + 4 * n16);
        xb[s] = *reinterpret_cast<const f4v *>(xext + c * kInLd + 64 + 4 * n16);
    }
}

// the batch's four k-steps into the 7 feature tiles: B = bfn(the lane's second float4, edge valid)
template <typename BFn>
__device__ __forceinline__ void mfma_batch(const f4v (&xa)[4], const f4v (&xb)[4], int32_t j0, int32_t deg, int kq,
                                           int n16, BFn &&bfn, f4v (&acc)[kInTiles]) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const bool ok = j0 + 4 * s + kq < deg;
        const float bv = bfn(xb[s], ok);
        acc[0] = mfma4(xa[s][0], bv, acc[0]);
        acc[1] = mfma4(xa[s][1], bv, acc[1]);
        acc[2] = mfma4(xa[s][2], bv, acc[2]);
        acc[3] = mfma4(xa[s][3], bv, acc[3]);
        // lanes 13..15 of the second float4 hold q (and lane 12's .yz zeros): not features
        const bool feat = n16 < 13;
        acc[4] = mfma4(feat ? xb[s][0] : 0.0f, bv, acc[4]);
        acc[5] = mfma4(feat ? xb[s][1] : 0.0f, bv, acc[5]);
        acc[6] = mfma4(feat ? xb[s][2] : 0.0f, bv, acc[6]);
    }
}

// One wave's walk over its rows (one per workgroup phase), software-pipelined so that a
// phase's barriers and projection do not drain the wave's memory pipeline: a row's next
// 16-edge batch is requested before the current one is summed, and the NEXT phase's row
// bounds (scalar loads), column window, row-local slot (`side`) and first batch are requested
// while this row is walked.  The cursor holds the current row; walk() advances it to `next`
// (-1: none).
struct RowCursor {
    int64_t e0 = 0;
    int32_t deg = 0, win = 0;
    float side = 0.0f;     // xext[row * 128 + side_slot]: aL (forward) / aR (backward) of the lane's head
    float side2 = 0.0f;    // xext[row * 128 + side_slot2] (side_slot2 >= 0): the forward's aR for T
    f4v xa[4], xb[4];      // the row's first batch (requested)
};

__device__ __forceinline__ void cursor_start(RowCursor &c, const int32_t *rowptr, const int32_t *col,
                                             const float *xext, int64_t row, int side_slot, int side_slot2, bool side_ok,
                                             int lane) {
    const int n16 = lane & 15, kq = lane >> 4;
    c.e0 = 0;
    c.deg = 0;
    c.side = 0.0f;
    c.side2 = 0.0f;
    if (row < 0) return;
    c.e0 = uniform(rowptr[row]);
    c.deg = uniform(rowptr[row + 1]) - (int32_t)c.e0;
    c.side = side_ok ? xext[row * kInLd + side_slot] : 0.0f;
    if (side_slot2 >= 0) c.side2 = side_ok ? xext[row * kInLd + side_slot2] : 0.0f;
    if (c.deg > 0) {
        c.win = col[c.e0 + (lane < c.deg ? lane : c.deg - 1)];
        load_batch(xext, c.win, 0, kq, n16, c.xa, c.xb);
    }
}

// body(xa, xb, j0, deg): the MFMA work of one loaded 16-edge batch
template <typename Body>
__device__ __forceinline__ void cursor_walk(RowCursor &c, const int32_t *rowptr, const int32_t *col,
                                            const float *xext, int64_t next, int side_slot, int side_slot2,
                                            bool side_ok, int lane, Body &&body) {
    const int n16 = lane & 15, kq = lane >> 4;
    // the next row's bounds: scalar loads (their own counter), waited for only below
    int64_t ne0 = 0;
    int32_t nend = 0;
    if (next >= 0) {
        const int64_t nx = __builtin_amdgcn_readfirstlane((int32_t)next);
        ne0 = rowptr[nx];
        nend = rowptr[nx + 1];
    }
    int32_t nwin = 0;
    float nside = 0.0f, nside2 = 0.0f;
    bool next_issued = false;
    auto issue_next = [&]() {
        if (next < 0 || next_issued) return;
        next_issued = true;
        const int32_t nd = nend - (int32_t)ne0;
        if (nd > 0) nwin = col[ne0 + (lane < nd ? lane : nd - 1)];
        nside = side_ok ? xext[next * kInLd + side_slot] : 0.0f;
        if (side_slot2 >= 0) nside2 = side_ok ? xext[next * kInLd + side_slot2] : 0.0f;
    };
    for (int32_t j0 = 0; j0 < c.deg; j0 += 16) {
        const int32_t j1 = j0 + 16;
        f4v ya[4], yb[4];
        const bool more = j1 < c.deg;
        if (more) {
            if ((j1 & 63) == 0) c.win = col[c.e0 + ((j1 + lane < c.deg) ? j1 + lane : c.deg - 1)];
            load_batch(xext, c.win, j1, kq, n16, ya, yb);
        }
        if (j0 == 0) issue_next();
        body(c.xa, c.xb, j0, c.deg);
        if (more) {
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                c.xa[s] = ya[s];
                c.xb[s] = yb[s];
            }
        }
    }
    issue_next();   // (an empty row walked no batch)
    c.e0 = uniform((int32_t)ne0);
    c.deg = next >= 0 ? uniform(nend - (int32_t)ne0) : 0;
    c.win = nwin;
    c.side = nside;
    c.side2 = nside2;
    if (c.deg > 0) load_batch(xext, c.win, 0, kq, n16, c.xa, c.xb);
}

// Forward.  Workgroup phase: wave w aggregates row order[8 blk + w] (B = p of head v for
// variant v < 8, m * p of head v - 8 for v >= 8), parks its tiles in LDS, then wave h
// projects the eight rows' head-h aggregates (M = 8 rows x {p, m p}, K = the 112 tile rows,
// N = D) with W_ext,h fragments held in registers.
// one workgroup of 8 waves per CU (2 per SIMD: ~210 VGPRs, no spills; 4 per SIMD spilled
// and ran 1.5x slower, tools/gat_input_bench.py)
// The forward's stash of the eight rows' aggregate tiles, in float4 units: tile t, k-quad kq,
// row slot s, variant v at ((t * 4 + kq) * 8 + s) * 16 + ((v + s) & 15).  The rotation by s
// puts a phase's stores (wave s: v = 0..15) and the projection's reads (wave h: the 16 (s, v)
// of head h) each on 16 distinct 16-B bank slots -- also across the k-quads that one
// ds_read_b128 lane group mixes (lanes {0-3, 12-15} of one quad, {4-11} of the next) -- where
// [slot][variant][tile][16] put the projection's 16 lanes on one bank (SQ_LDS_BANK_CONFLICT:
// 71 % of the kernel's LDS cycles, profiles/r06_lds_conflicts.txt).
__device__ __forceinline__ int fwd_stash(int t, int kq, int s, int v) {
    return ((t * 4 + kq) * kInWaves + s) * 16 + ((v + s) & 15);
}

// T mode (TM, symmetric pattern): the same walk also forms the backward's per-column
// aggregates T_h[c] = sum_{r in N(c)} alpha_{r->c},h Xin_ext[r], alpha = p(aL[r] + aR[c]) q[r]
// (the gathered row carries aL[r] and q[r], the latter from k_gat_in_q), so the backward reads
// T instead of gathering the extended rows a second time.  Row c's T tiles go to
// T[((c * 7 + t) * 4 + kq) * 8 + head] (float4s: 896 floats per row).
template <bool TM>
__global__ __launch_bounds__(kInBlock, 2) void k_gat_in_fwd(InFwdParams p) {
    __shared__ f4v stash[kInWaves * 16 * kInTiles * 4];   // fwd_stash
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, n16 = lane & 15, kq = lane >> 4;
    const int h = wave;
    // B fragments of the projection: W_ext,h[j = 16 nt + n16][feature(t, 4 kq + q4)]
    float wf[kInTiles][4][2];
#pragma unroll
    for (int t = 0; t < kInTiles; ++t)
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) {
                const int j = 16 * nt + n16, f = tile_feature(t, 4 * kq + q4, p.fin);
                float v = 0.0f;
                if (h < p.H && j < p.D) {
                    const int64_t o = (int64_t)h * p.D + j;
                    if (f >= 0) v = p.W[o * p.ldw + f];
                    else if (f == -2) v = p.b ? p.b[o] : 0.0f;
                }
                wf[t][q4][nt] = v;
            }
    const float *stf = reinterpret_cast<const float *>(stash);
    const int64_t nblk = (p.n_rows + kInWaves - 1) / kInWaves;
    auto row_of = [&](int64_t b) -> int64_t {
        const int64_t ri = b * kInWaves + wave;
        if (b >= nblk || ri >= p.n_rows) return -1;
        return p.order ? (int64_t)__builtin_amdgcn_readfirstlane(p.order[ri]) : ri;
    };
    const bool side_ok = n16 < p.H;
    const int side2 = TM ? aR_slot(n16 & 7) : -1;
    // T mode: q[h] of a gathered row from lane 13 + h / 3 of its edge's 16 lanes, component h % 3
    const int hq = n16 & 7;
    const int qsrc = (16 * kq + 13 + hq / 3) * 4, qc = hq % 3;
    RowCursor cur;
    cursor_start(cur, p.rowptr, p.col, p.xext, row_of(blockIdx.x), aL_slot(n16 & 7), side2, side_ok, lane);
    for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
        f4v acc[kInTiles], accT[kInTiles];
#pragma unroll
        for (int t = 0; t < kInTiles; ++t) acc[t] = accT[t] = f4v{0.0f, 0.0f, 0.0f, 0.0f};
        const int64_t myrow = TM ? row_of(blk) : -1;
        // the rows this lane's projection outputs will go to (slots 2 kq, 2 kq + 1), requested
        // before the walk so the stores after the barrier wait on nothing
        int64_t prow[2];
#pragma unroll
        for (int hs = 0; hs < 2; ++hs) {
            const int64_t si = blk * kInWaves + 2 * kq + hs;
            prow[hs] = si < p.n_rows ? (p.order ? (int64_t)p.order[si] : si) : -1;
        }
        {
            const float al = cur.side, ar = cur.side2;
            const int H = p.H;
            const float slope = p.slope;
            auto bfn = [&](const f4v &xb, bool ok) {
                const float t = __fadd_rn(al, xb[3]);   // lanes v < 8: aR[col][v]
                const bool pos = t > 0.0f;
                float pv = ref_exp(pos ? t : __fmul_rn(t, slope));
                if (!(ok && n16 < H)) pv = 0.0f;
                const float mp = pos ? pv : __fmul_rn(pv, slope);
                const float mpo = ror8(mp);
                return n16 < 8 ? pv : mpo;
            };
            // the backward's alpha of edge (col -> row): gala_gat_in_bwd's formula
            auto bfnT = [&](const f4v &xb, bool ok) {
                const float alr = ror8(xb[3]);            // aL[col][v] from lane v + 8
                const float q0 = __int_as_float(__builtin_amdgcn_ds_bpermute(qsrc, __float_as_int(xb[0])));
                const float q1 = __int_as_float(__builtin_amdgcn_ds_bpermute(qsrc, __float_as_int(xb[1])));
                const float q2 = __int_as_float(__builtin_amdgcn_ds_bpermute(qsrc, __float_as_int(xb[2])));
                const float qr = qc == 0 ? q0 : (qc == 1 ? q1 : q2);
                const float t = __fadd_rn(alr, ar);
                const float pv = ref_exp(t > 0.0f ? t : __fmul_rn(t, slope));
                const float a = __fmul_rn(pv, qr);
                return (ok && n16 < H) ? a : 0.0f;
            };
            cursor_walk(cur, p.rowptr, p.col, p.xext, row_of(blk + gridDim.x), aL_slot(n16 & 7), side2, side_ok, lane,
                        [&](const f4v (&xa)[4], const f4v (&xb)[4], int32_t j0, int32_t deg) {
                            mfma_batch(xa, xb, j0, deg, kq, n16, bfn, acc);
                            if (TM) mfma_batch(xa, xb, j0, deg, kq, n16, bfnT, accT);
                        });
        }
        if (TM && myrow >= 0 && n16 < kInMaxHeads) {
            f4v *tr = reinterpret_cast<f4v *>(p.T) + myrow * (kInTiles * 4 * kInMaxHeads);
#pragma unroll
            for (int t = 0; t < kInTiles; ++t) tr[(t * 4 + kq) * kInMaxHeads + n16] = accT[t];
        }
#pragma unroll
        for (int t = 0; t < kInTiles; ++t) stash[fwd_stash(t, kq, wave, n16)] = acc[t];
        __syncthreads();
        if (h < p.H) {
            f4v y[2] = {f4v{0.0f, 0.0f, 0.0f, 0.0f}, f4v{0.0f, 0.0f, 0.0f, 0.0f}};
            const int s_a = n16 >> 1, v_a = h + 8 * (n16 & 1);
#pragma unroll
            for (int t = 0; t < kInTiles; ++t) {
                const f4v a4 = stash[fwd_stash(t, kq, s_a, v_a)];
#pragma unroll
                for (int q4 = 0; q4 < 4; ++q4) {
                    y[0] = mfma4(a4[q4], wf[t][q4][0], y[0]);
                    y[1] = mfma4(a4[q4], wf[t][q4][1], y[1]);
                }
            }
            // D[m = 4 kq + i][n16]: slot s = m / 2, variant class u = m % 2
#pragma unroll
            for (int hs = 0; hs < 2; ++hs) {
                const int s = 2 * kq + hs;
                const int64_t row = prow[hs];
                if (row < 0) continue;
                // sum p / sum m p: tile 4, float 12 (k-quad 3, component 0) of variants h, h + 8
                const float S = stf[fwd_stash(4, 3, s, h) * 4];
                const float Sm = stf[fwd_stash(4, 3, s, h + 8) * 4];
                // REF: 1 / (1e-12 + sum p); T mode: k_gat_in_q's (the sequential row sum)
                const float qv = TM ? p.xext[row * kInLd + q_slot(h)] : 1.0f / __fadd_rn(S, 1e-12f);
#pragma unroll
                for (int nt = 0; nt < 2; ++nt) {
                    const int j = 16 * nt + n16;
                    if (j >= p.D) continue;
                    const int64_t o = row * p.ldy + (int64_t)h * p.D + j;
                    const float yv = __fmul_rn(qv, y[nt][2 * hs]);
                    // torch::relu keeps NaN (clamp_min); its backward zeroes it (out > 0 fails)
                    p.Y[o] = (!p.relu || yv > 0.0f || yv != yv) ? yv : 0.0f;
                    p.Ym[o] = __fmul_rn(qv, y[nt][2 * hs + 1]);
                }
                if (n16 == 0) {
                    p.q[row * p.H + h] = qv;
                    p.sma[row * p.H + h] = __fmul_rn(qv, Sm);
                    if (!TM) p.xext[row * kInLd + q_slot(h)] = qv;
                }
            }
        }
        __syncthreads();
    }
}

struct InBwdParams {
    const int32_t *rowptr, *col, *order;   // the transposed pattern
    int64_t n_rows;
    const float *xext, *dY, *Y, *Ym, *sma;
    int64_t ldy;
    int32_t fin, H, D;
    float slope;
    float *daL;
    float *part;
    int32_t relu;   // Y holds relu(the aggregation): dY is masked by Y > 0 (torch's threshold_backward)    // [gridDim][H][2][kInTiles][64][4]
    const float *T; // T mode: the forward's per-column aggregates (no walk over the pattern)
};

template <int DW>   // lanes per head in the row-local d_aL dots: D / 4
__device__ __forceinline__ float head_dot_sum(float v) { return group_sum<DW>(v); }

// Backward.  Workgroup phase: wave w walks column c = order[8 blk + w] of the transposed
// pattern (the rows r whose edge e = (r -> c) it holds), accumulates T_h[c] = sum alpha_e,h
// Xin_ext[r] (alpha rebuilt from aL[r], q[r] in r's extended row and aR[c]) and c's d_aL from
// the forward's row statistics; then wave h adds dY_h[c]^T T_h[c] of the eight columns into
// its register accumulators M_h[D x 112] (K = the columns).  Partials per workgroup.
// The backward's stash, in floats: slot s, head h, tile t, element i at s * kBwdSlot + h * kBwdHead
// + t * 16 + i -- the 4-float pads put a phase's float4 stores (wave s, lanes h = 0..7 of one
// k-quad) and the M phase's reads (lanes of two k-quads: slots s, s + 1) on distinct banks; the
// columns' dY at slot * kDyLd floats likewise (unpadded: 2-way conflicts on every read).
constexpr int kBwdHead = kInTiles * 16 + 4;             // 116 floats
constexpr int kBwdSlot = kInMaxHeads * kBwdHead + 16;   // 944 floats: slots s, s + 1 16 banks apart
constexpr int kDyLd = 4 * (kWave + 4);                  // 272 floats of dY per slot

template <int DW, bool TM>
__global__ __launch_bounds__(kInBlock, 2) void k_gat_in_bwd(InBwdParams p) {
    __shared__ f4v stash[kInWaves * kBwdSlot / 4];   // see kBwdSlot
    __shared__ f4v dstash[kInWaves * kDyLd / 4];     // [slot][kDyLd]: the columns' dY (masked)
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, n16 = lane & 15, kq = lane >> 4;
    const int h = wave;
    const float *stf = reinterpret_cast<const float *>(stash);
    f4v M[2][kInTiles];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int t = 0; t < kInTiles; ++t) M[mt][t] = f4v{0.0f, 0.0f, 0.0f, 0.0f};
    const int F = p.H * p.D;
    const int64_t nblk = (p.n_rows + kInWaves - 1) / kInWaves;
    // q[h] of a gathered row: lane 13 + h / 3 of its edge's 16 lanes, component h % 3
    const int hq = n16 & 7;
    const int qsrc = (16 * kq + 13 + hq / 3) * 4, qc = hq % 3;
    auto col_of = [&](int64_t b) -> int64_t {
        const int64_t ci = b * kInWaves + wave;
        if (b >= nblk || ci >= p.n_rows) return -1;
        return p.order ? (int64_t)__builtin_amdgcn_readfirstlane(p.order[ci]) : ci;
    };
    const bool side_ok = n16 < p.H;
    RowCursor cur;
    if (!TM) cursor_start(cur, p.rowptr, p.col, p.xext, col_of(blockIdx.x), aR_slot(n16 & 7), -1, side_ok, lane);
    for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
        f4v acc[kInTiles];
#pragma unroll
        for (int t = 0; t < kInTiles; ++t) acc[t] = f4v{0.0f, 0.0f, 0.0f, 0.0f};
        const int64_t c = col_of(blk);
        // the column's row statistics for d_aL, requested before the walk (F = H*D <= 256:
        // one float4 per lane)
        const int f = 4 * lane;
        f4v dy = f4v{0.0f, 0.0f, 0.0f, 0.0f}, yy = dy, ym = dy;
        if (c >= 0 && f < F) {
            dy = *reinterpret_cast<const f4v *>(p.dY + c * p.ldy + f);
            yy = *reinterpret_cast<const f4v *>(p.Y + c * p.ldy + f);
            ym = *reinterpret_cast<const f4v *>(p.Ym + c * p.ldy + f);
            if (p.relu) {
#pragma unroll
                for (int i = 0; i < 4; ++i) dy[i] = yy[i] > 0.0f ? dy[i] : 0.0f;
            }
        }
        if (TM) {   // the forward's T tiles of column c (k_gat_in_fwd<true>)
            if (c >= 0 && n16 < kInMaxHeads) {
                const f4v *tr = reinterpret_cast<const f4v *>(p.T) + c * (kInTiles * 4 * kInMaxHeads);
#pragma unroll
                for (int t = 0; t < kInTiles; ++t) acc[t] = tr[(t * 4 + kq) * kInMaxHeads + n16];
            }
        } else {
            const float ar = cur.side;
            const int H = p.H;
            const float slope = p.slope;
            auto bfn = [&](const f4v &xb, bool ok) {
                const float alr = ror8(xb[3]);            // aL[r][v] from lane v + 8
                const float q0 = __int_as_float(__builtin_amdgcn_ds_bpermute(qsrc, __float_as_int(xb[0])));
                const float q1 = __int_as_float(__builtin_amdgcn_ds_bpermute(qsrc, __float_as_int(xb[1])));
                const float q2 = __int_as_float(__builtin_amdgcn_ds_bpermute(qsrc, __float_as_int(xb[2])));
                const float qr = qc == 0 ? q0 : (qc == 1 ? q1 : q2);
                const float t = __fadd_rn(alr, ar);
                const float pv = ref_exp(t > 0.0f ? t : __fmul_rn(t, slope));
                const float a = __fmul_rn(pv, qr);       // K8: alpha = p * q[row]
                return (ok && n16 < H) ? a : 0.0f;
            };
            cursor_walk(cur, p.rowptr, p.col, p.xext, col_of(blk + gridDim.x), aR_slot(n16 & 7), -1, side_ok, lane,
                        [&](const f4v (&xa)[4], const f4v (&xb)[4], int32_t j0, int32_t deg) {
                            mfma_batch(xa, xb, j0, deg, kq, n16, bfn, acc);
                        });
        }
        if (c >= 0) {   // d_aL[c] from the forward's row statistics (gala_gat_bwd_stats_f32's formula)
            float syy = 0.0f, sym = 0.0f;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                syy = fmaf(dy[i], yy[i], syy);
                sym = fmaf(dy[i], ym[i], sym);
            }
            syy = head_dot_sum<DW>(syy);
            sym = head_dot_sum<DW>(sym);
            if (f < F && (f % p.D) == 0) {
                const int hh = f / p.D;
                const float accv = syy + 1e-12f;                       // K7 on sds (common.h:793-794)
                p.daL[c * p.H + hh] = (sym - accv * p.sma[c * p.H + hh]) + 1e-12f;   // common.h:662-667
            }
        }
        dstash[wave * (kDyLd / 4) + lane] = dy;   // the M phase's A operand, from LDS after the barrier
        if (n16 < kInMaxHeads) {
#pragma unroll
            for (int t = 0; t < kInTiles; ++t) stash[(wave * kBwdSlot + n16 * kBwdHead + t * 16) / 4 + kq] = acc[t];
        }
        __syncthreads();
        if (h < p.H) {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const int s = 4 * ks + kq;
                const int64_t si = blk * kInWaves + s;
                const bool ok = si < p.n_rows;
                const float *dsf = reinterpret_cast<const float *>(dstash) + s * kDyLd;
                float a[2];
#pragma unroll
                for (int mt = 0; mt < 2; ++mt) {
                    const int j = 16 * mt + n16;
                    a[mt] = (ok && j < p.D) ? dsf[h * p.D + j] : 0.0f;
                }
#pragma unroll
                for (int t = 0; t < kInTiles; ++t) {
                    const float bv = ok ? stf[s * kBwdSlot + h * kBwdHead + t * 16 + n16] : 0.0f;
                    M[0][t] = mfma4(a[0], bv, M[0][t]);
                    M[1][t] = mfma4(a[1], bv, M[1][t]);
                }
            }
        }
        __syncthreads();
    }
    if (h < p.H) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int t = 0; t < kInTiles; ++t)
                *reinterpret_cast<f4v *>(p.part + (((((int64_t)blockIdx.x * p.H + h) * 2 + mt) * kInTiles + t) * 64 +
                                                   lane) * 4) = M[mt][t];
    }
}

// M[h][j][k], k < fin a feature, k = fin the ones column: the workgroups' partials summed
__global__ __launch_bounds__(kBlock) void k_gat_in_reduce(const float *part, int32_t nparts, int32_t H, int32_t D,
                                                          int32_t fin, float *M) {
    const int64_t id = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t per = (int64_t)H * 2 * kInTiles * 64 * 4;
    if (id >= per) return;
    const int i = id & 3, lane = (int)((id >> 2) & 63);
    const int64_t rest = id >> 8;
    const int t = (int)(rest % kInTiles), mt = (int)((rest / kInTiles) % 2), h = (int)(rest / (kInTiles * 2));
    const int j = 16 * mt + 4 * (lane >> 4) + i;
    const int f = tile_feature(t, lane & 15, fin);
    if (j >= D || f == -1) return;
    float s = 0.0f;
    for (int b = 0; b < nparts; ++b) s += part[(int64_t)b * per + id];
    M[((int64_t)h * D + j) * (fin + 1) + (f == -2 ? fin : f)] = s;
}

// T mode's row sums before the forward: q_h[r] = 1 / (1e-12 + sum_e p(aL[r] + aR[c_e])) for every
// row (the forward's T tiles read q of the rows they gather), 8 lanes per row (lane = head),
// each summing its head's p over the row's edges in CSR order -- the reference's sequential
// row sum (K7) -- into the row's q slots of the extended table.
// the rows' aR in a compact [n][8] table (78 MB at the Products shape: the q pass's gathers
// hit the MALL instead of fetching a 128-B line of the 1.25 GB extended table per edge)
__global__ __launch_bounds__(kBlock) void k_gat_in_ar(const float *xext, int64_t n_rows, float *ar) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n_rows * 8) ar[i] = xext[(i >> 3) * kInLd + aR_slot((int)(i & 7))];
}

__global__ __launch_bounds__(kBlock) void k_gat_in_q(const int32_t *rowptr, const int32_t *col, int64_t n_rows,
                                                     int32_t H, float slope, const float *art, float *xext) {
    const int h = threadIdx.x & 7;
    const int64_t g0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 3, gstep = ((int64_t)gridDim.x * kBlock) >> 3;
    for (int64_t r = g0; r < n_rows; r += gstep) {
        if (h >= H) continue;
        const int64_t e0 = rowptr[r], e1 = rowptr[r + 1];
        const float al = xext[r * kInLd + aL_slot(h)];
        float S = 0.0f;
        // 8 edges per step, the next step's column indices requested before this step's sums
        constexpr int U = 8;
        int32_t cn[U];
#pragma unroll
        for (int k = 0; k < U; ++k) cn[k] = e0 + k < e1 ? col[e0 + k] : 0;
        for (int64_t e = e0; e < e1; e += U) {
            float ar[U];
#pragma unroll
            for (int k = 0; k < U; ++k) ar[k] = art[(int64_t)cn[k] * 8 + h];
#pragma unroll
            for (int k = 0; k < U; ++k) cn[k] = e + U + k < e1 ? col[e + U + k] : 0;
#pragma unroll
            for (int k = 0; k < U; ++k) {
                if (e + k < e1) {
                    const float t = __fadd_rn(al, ar[k]);
                    S = __fadd_rn(S, ref_exp(t > 0.0f ? t : __fmul_rn(t, slope)));
                }
            }
        }
        xext[r * kInLd + q_slot(h)] = 1.0f / __fadd_rn(S, 1e-12f);
    }
}

int grid_for(int64_t n_rows) {
    const int64_t nblk = (n_rows + kInWaves - 1) / kInWaves;
    return (int)std::min<int64_t>(std::max<int64_t>(nblk, 1), kInGrid);
}

int check_in_graph(const gala_csr_t *A, int32_t fin, int32_t heads, int32_t D) {
    int st = check_csr(A);
    if (st) return st;
    if (fin < 1 || heads < 1 || D < 1) return GALA_ERR_INVALID_ARG;
    // the extended row holds at most 100 features and 8 heads; the projection's N = D <= 32
    // with D / 4 lanes per head in the d_aL dots; one segment, a square pattern, no hub-row
    // plan (a hub row is one wave's serial walk: those graphs stay on the statistics pair)
    if (fin > kInMaxFin || heads > kInMaxHeads || !(D == 4 || D == 8 || D == 16 || D == 32) || A->n_seg != 1 ||
        A->n_rows != A->n_cols || (A->split && A->split->n_rows_split > 0))
        return GALA_ERR_UNSUPPORTED;
    return GALA_OK;
}

}  // namespace

extern "C" int gala_gat_in_prep_f32(int64_t n, int32_t fin, const float *Xin, int64_t ldxin, int32_t heads,
                                    const float *u, const float *c, float *Xext, void *stream) {
    if (n < 0 || fin < 1 || heads < 1 || ldxin < fin) return GALA_ERR_INVALID_ARG;
    if (fin > kInMaxFin || heads > kInMaxHeads) return GALA_ERR_UNSUPPORTED;
    if (n == 0) return GALA_OK;
    if (!Xin || !u || !c || !Xext || ((uintptr_t)Xext & 15)) return GALA_ERR_INVALID_ARG;
    InPrepParams p{Xin, n, ldxin, fin, heads, u, c, Xext};
    const int64_t groups = (n + kBlock / 16 - 1) / (kBlock / 16);
    hipLaunchKernelGGL(k_gat_in_prep, dim3((unsigned)std::min<int64_t>(groups, 4096)), dim3(kBlock), 0,
                       (hipStream_t)stream, p);
    return launch_status();
}

namespace {
int fwd_launch(const gala_csr_t *A, const int32_t *order, int32_t fin, int32_t heads, int32_t D, float slope,
               float *Xext, const float *W, int64_t ldw, const float *b, float *Y, float *Ym, int64_t ldy, float *q,
               float *sma, int32_t flags, float *T, void *stream) {
    int st = check_in_graph(A, fin, heads, D);
    if (st) return st;
    if (ldw < fin || ldy < (int64_t)heads * D || (flags & ~GALA_GAT_IN_RELU)) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0) return GALA_OK;
    if (!Xext || !W || !Y || !Ym || !q || !sma || ((uintptr_t)Xext & 15) || ((uintptr_t)T & 15))
        return GALA_ERR_INVALID_ARG;
    InFwdParams p{A->rowptr, A->col, order ? order : (A->split ? A->split->row_order : nullptr), A->n_rows, Xext, W,
                  b, ldw,
                  fin, heads, D, slope, Y, Ym, q, sma, ldy, (flags & GALA_GAT_IN_RELU) ? 1 : 0, T};
    hipStream_t hs = (hipStream_t)stream;
    if (T) {
        // T's first 8 n floats hold the compact aR table until the forward writes T
        hipLaunchKernelGGL(k_gat_in_ar, dim3((unsigned)((A->n_rows * 8 + kBlock - 1) / kBlock)), dim3(kBlock), 0, hs,
                           Xext, A->n_rows, T);
        if ((st = launch_status())) return st;
        const int64_t groups = (A->n_rows + kBlock / 8 - 1) / (kBlock / 8);
        hipLaunchKernelGGL(k_gat_in_q, dim3((unsigned)std::min<int64_t>(groups, 8192)), dim3(kBlock), 0, hs,
                           A->rowptr, A->col, A->n_rows, heads, slope, T, Xext);
        if ((st = launch_status())) return st;
        hipLaunchKernelGGL(k_gat_in_fwd<true>, dim3(grid_for(A->n_rows)), dim3(kInBlock), 0, hs, p);
    } else {
        hipLaunchKernelGGL(k_gat_in_fwd<false>, dim3(grid_for(A->n_rows)), dim3(kInBlock), 0, hs, p);
    }
    return launch_status();
}
}  // namespace

extern "C" int gala_gat_in_fwd_f32(const gala_csr_t *A, const int32_t *order, int32_t fin, int32_t heads, int32_t D,
                                   float slope,
                                   float *Xext, const float *W, int64_t ldw, const float *b, float *Y, float *Ym,
                                   int64_t ldy, float *q, float *sma, int32_t flags, void *stream) {
    return fwd_launch(A, order, fin, heads, D, slope, Xext, W, ldw, b, Y, Ym, ldy, q, sma, flags, nullptr, stream);
}

extern "C" int gala_gat_in_fwd_t_f32(const gala_csr_t *A, const int32_t *order, int32_t fin, int32_t heads, int32_t D,
                                     float slope, float *Xext, const float *W, int64_t ldw, const float *b, float *Y,
                                     float *Ym, int64_t ldy, float *q, float *sma, int32_t flags, float *T,
                                     void *stream) {
    if (!T) return GALA_ERR_INVALID_ARG;
    return fwd_launch(A, order, fin, heads, D, slope, Xext, W, ldw, b, Y, Ym, ldy, q, sma, flags, T, stream);
}

extern "C" int64_t gala_gat_in_bwd_workspace(int32_t heads) {
    if (heads < 1 || heads > kInMaxHeads) return -1;
    return (int64_t)kInGrid * heads * 2 * kInTiles * 64 * 4 * (int64_t)sizeof(float);
}

namespace {
// AT: the transposed pattern (walked), or null with T: the forward's T tiles of n_rows columns
int bwd_launch(const gala_csr_t *AT, int64_t n_rows, const int32_t *order, int32_t fin, int32_t heads, int32_t D,
               float slope, const float *Xext, const float *T, const float *dY, const float *Y, const float *Ym,
               int64_t ldy, const float *sma, float *daL, float *M, void *ws_, int64_t ws_bytes, int32_t flags,
               void *stream) {
    float *ws = (float *)ws_;
    int st;
    if (AT) {
        if ((st = check_in_graph(AT, fin, heads, D))) return st;
        n_rows = AT->n_rows;
    } else {
        if (n_rows < 0 || fin < 1 || heads < 1 || D < 1) return GALA_ERR_INVALID_ARG;
        if (fin > kInMaxFin || heads > kInMaxHeads || !(D == 4 || D == 8 || D == 16 || D == 32))
            return GALA_ERR_UNSUPPORTED;
    }
    if (ldy < (int64_t)heads * D || (ldy & 3) || (flags & ~GALA_GAT_IN_RELU)) return GALA_ERR_INVALID_ARG;
    if (!M) return GALA_ERR_INVALID_ARG;
    hipStream_t hs = (hipStream_t)stream;
    const int64_t outn = (int64_t)heads * D * (fin + 1);
    if (n_rows == 0) {
        return hipMemsetAsync(M, 0, outn * sizeof(float), hs) == hipSuccess ? GALA_OK : GALA_ERR_HIP;
    }
    if ((AT ? (!Xext || ((uintptr_t)Xext & 15)) : (!T || ((uintptr_t)T & 15))) || !dY || !Y || !Ym || !sma || !daL ||
        !ws || ((uintptr_t)dY & 15) || ((uintptr_t)Y & 15) || ((uintptr_t)Ym & 15))
        return GALA_ERR_INVALID_ARG;
    if (ws_bytes < gala_gat_in_bwd_workspace(heads)) return GALA_ERR_INVALID_ARG;
    const int grid = grid_for(n_rows);
    const int32_t *ord = order ? order : (AT && AT->split ? AT->split->row_order : nullptr);
    InBwdParams p{AT ? AT->rowptr : nullptr, AT ? AT->col : nullptr, ord, n_rows, Xext, dY, Y, Ym,
                  sma, ldy, fin, heads, D, slope, daL, ws, (flags & GALA_GAT_IN_RELU) ? 1 : 0, T};
    if (hipMemsetAsync(M, 0, outn * sizeof(float), hs) != hipSuccess) return GALA_ERR_HIP;
#define GALA_IN_BWD(DW)                                                                           \
    do {                                                                                          \
        if (AT) hipLaunchKernelGGL((k_gat_in_bwd<DW, false>), dim3(grid), dim3(kInBlock), 0, hs, p); \
        else hipLaunchKernelGGL((k_gat_in_bwd<DW, true>), dim3(grid), dim3(kInBlock), 0, hs, p);     \
    } while (0)
    switch (D / 4) {
    case 1: GALA_IN_BWD(1); break;
    case 2: GALA_IN_BWD(2); break;
    case 4: GALA_IN_BWD(4); break;
    default: GALA_IN_BWD(8); break;
    }
#undef GALA_IN_BWD
    st = launch_status();
    if (st) return st;
    const int64_t per = (int64_t)heads * 2 * kInTiles * 64 * 4;
    hipLaunchKernelGGL(k_gat_in_reduce, dim3((unsigned)((per + kBlock - 1) / kBlock)), dim3(kBlock), 0, hs,
                       (const float *)ws, grid, heads, D, fin, M);
    return launch_status();
}
}  // namespace

extern "C" int gala_gat_in_bwd_f32(const gala_csr_t *AT, const int32_t *order, int32_t fin, int32_t heads, int32_t D,
                                   float slope,
                                   const float *Xext, const float *dY, const float *Y, const float *Ym,
                                   int64_t ldy, const float *sma, float *daL, float *M, void *ws_,
                                   int64_t ws_bytes, int32_t flags, void *stream) {
    if (!AT) return GALA_ERR_INVALID_ARG;
    return bwd_launch(AT, 0, order, fin, heads, D, slope, Xext, nullptr, dY, Y, Ym, ldy, sma, daL, M, ws_, ws_bytes,
                      flags, stream);
}

extern "C" int gala_gat_in_bwd_t_f32(int64_t n_rows, const int32_t *order, int32_t fin, int32_t heads, int32_t D,
                                     const float *T, const float *dY, const float *Y, const float *Ym, int64_t ldy,
                                     const float *sma, float *daL, float *M, void *ws_, int64_t ws_bytes,
                                     int32_t flags, void *stream) {
    return bwd_launch(nullptr, n_rows, order, fin, heads, D, 0.0f, nullptr, T, dY, Y, Ym, ldy, sma, daL, M, ws_,
                      ws_bytes, flags, stream);
}

}  // namespace gala
