// SpMM neighbour aggregation for gfx950 (CDNA4, wave64).
//
// Replaces the emitted `aggregate_node_mul_sum[_direct]_coarse{C}_kernel{k}[_offset]`
// family (src/codegen/cuda.h:286-436) and its launch tree (coarsenedKernelCall,
// cuda.h:58-168), the cuSPARSE "gather_forward" path (cuda.h:211-279) and the
// kernel-sampled variants (cuda.h:313-321,389-397).
//
// Layout of one launch: a "row group" of G lanes (G a power of two) owns one CSR row;
// lane g of the group owns VEC contiguous fp32 features at column (ch*G + g)*VEC for
// ch < CH, so the group reads whole X rows with VEC*4-byte coalesced loads
// (F = 32 -> float4 x 8 lanes = one 128-B line per neighbour).  A wave holds 64/G rows.
// Inside a row, edges are accumulated sequentially in CSR order (segment 0 first),
// with the neighbour loads of U edges issued before the first add, so the result is
// bit-identical to the reference kernel while each lane keeps U*CH vector loads in
// flight.  All address arithmetic is 64-bit.
#include <stddef.h>
#include <cstdlib>

#include "gala_internal.h"

namespace gala {

template <int VEC>
struct VecT;
template <>
struct VecT<1> {
    typedef float T;
};
template <>
struct VecT<2> {
    typedef float T __attribute__((ext_vector_type(2)));
};
template <>
struct VecT<4> {
    typedef float T __attribute__((ext_vector_type(4)));
};

struct SpmmParams {
    const int32_t *rowptr;
    const int32_t *col;
    const float *val;
    const float *val_rs;      // nullable [n_rows * val_heads]: w_e = val[e,h] * val_rs[row,h]
    const float *X;
    float *Y;
    const float *src_scale;
    const float *dst_scale;
    int64_t n_rows;
    int64_t ldx;
    int64_t ldy;
    int32_t F;
    int32_t val_heads;
    int32_t head_dim;   // F / val_heads
    int32_t accum;      // 1: Y += ..., 0: Y = ...
    int32_t nsamp, ra, rb;
    int32_t split_threshold;  // > 0: rows longer than this are left to the split kernels
    const int32_t *row_order; // nullable: row group i handles row row_order[i]
    int32_t xcd_order;        // 1: XCD-aware block order (logical_block_runs)
    int32_t dst_deg;          // 1: the dst factor is 1/sqrt(deg) of the row (one segment)
    float *Y2;                // nullable epilogue output: Y2[r] = s2[r] * Y[r]
    int64_t ldy2;
    const float *y2_scale;    // s2 (NULL: the dst factor)
    // ABI 4 epilogue fields (gala_spmm_epilogue_t): the ReLU prologue's act (RELU kernels:
    // the gathered source is src_scale[c] * relu(src_act[c] * X[c])), and the ReLU-backward
    // epilogue (relu_x != NULL: Y[r] = relu_act[r] * (relu(relu_act[r] * relu_x[r]) <= 0 ? 0 : Y[r]))
    int32_t relu_prologue;
    const float *src_act;
    const float *relu_x;
    int64_t ldrx;
    const float *relu_act;
    SegTable seg;
};

// torch.relu as its GPU kernel computes it: t > 0 ? t : +0, NaN passes
__device__ __forceinline__ float relu_t(float t) { return (t > 0.0f || t != t) ? t : 0.0f; }

// GCN norm deg^-0.5 of a row count: the expression of k_degree_count (power -0.5), so an
// in-kernel norm is bit-identical to the degree pass's
__device__ __forceinline__ float deg_rsqrt(float d) { return 1.0f / sqrtf(d); }

// the dst factor of `row` (has: whether there is one)
__device__ __forceinline__ float dst_factor(const SpmmParams &p, int64_t row, bool &has) {
    has = p.dst_deg || p.dst_scale;
    if (p.dst_deg) return deg_rsqrt((float)(p.rowptr[row + 1] - p.rowptr[row]));
    return p.dst_scale ? p.dst_scale[row] : 1.0f;
}

template <int VEC>
__device__ __forceinline__ typename VecT<VEC>::T ldv(const float *p) {
    return *reinterpret_cast<const typename VecT<VEC>::T *>(p);
}
template <int VEC>
__device__ __forceinline__ void stv(float *p, typename VecT<VEC>::T v) {
    *reinterpret_cast<typename VecT<VEC>::T *>(p) = v;
}

// element access helpers for ext_vector / scalar
template <int VEC>
__device__ __forceinline__ float &el(typename VecT<VEC>::T &v, int i) {
    return reinterpret_cast<float *>(&v)[i];
}

// acc (+)= w * (s * x), reference rounding:  s*x is the torch `norm * res` product
// (rounded), `local + A*B` is contracted to fma by nvcc (cuda.h:335-342).
// RELU: the next layer's ReLU prologue on the gathered element, v = s * relu(a * x) with the
// roundings of gala_row_scale_relu_f32 (a, s = 1.0f when absent: exact)
template <int VEC, bool W, bool SRCS, bool RELU = false>
__device__ __forceinline__ void accumulate(typename VecT<VEC>::T &acc,
                                           const typename VecT<VEC>::T &x, float w, float s,
                                           float a = 1.0f) {
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
        float v = reinterpret_cast<const float *>(&x)[i];
        if (RELU) v = relu_t(__fmul_rn(a, v));
        if (SRCS) v = __fmul_rn(s, v);
        float &r = el<VEC>(acc, i);
        if (W)
            r = fmaf(w, v, r);
        else
            r = __fadd_rn(r, v);
    }
}

// Per-lane column ownership of a row group.  When F is not a multiple of VEC the rows are
// padded (ldx, ldy >= F rounded up to VEC, checked on the host): the last vector of a row
// loads the padding too (never used) and stores only its nv < VEC real columns.
template <int VEC, int G, int CH, bool W>
struct Cols {
    bool valid[CH];
    int64_t off[CH];
    int head[CH];
    int nv[CH];
    __device__ __forceinline__ Cols(const SpmmParams &p, int gl) {
#pragma unroll
        for (int ch = 0; ch < CH; ++ch) {
            const int f = (ch * G + gl) * VEC;
            valid[ch] = f < p.F;  // lanes past F load a valid column and never store
            off[ch] = valid[ch] ? f : 0;
            head[ch] = W ? (int)(off[ch] / p.head_dim) : 0;
            nv[ch] = valid[ch] ? (p.F - f < VEC ? p.F - f : VEC) : 0;
        }
    }
};

// Y row slice store of nv <= VEC columns (nv < VEC only for a padded row's last vector).
template <int VEC>
__device__ __forceinline__ void stv_n(float *p, const typename VecT<VEC>::T &v, int nv) {
    if (nv == VEC) {
        stv<VEC>(p, v);
        return;
    }
#pragma unroll
    for (int i = 0; i < VEC; ++i)
        if (i < nv) p[i] = reinterpret_cast<const float *>(&v)[i];
}

// acc += the edges [e0, e1) of one row (or nsamp kernel samples), sequentially in CSR
// order; the loads of U edges are issued before the first add of the batch.
template <int VEC, int G, int CH, int U, bool W, bool SAMP, bool SRCS, bool RELU = false>
__device__ __forceinline__ void accumulate_range(const SpmmParams &p, const Cols<VEC, G, CH, W> &cl,
                                                 int64_t row, int64_t e0, int64_t e1,
                                                 typename VecT<VEC>::T (&acc)[CH]) {
    typedef typename VecT<VEC>::T V;
    const int32_t deg = (int32_t)(e1 - e0);
    const int32_t n = SAMP ? (deg > 0 ? p.nsamp : 0) : deg;
    // factored edge values (the GAT forward's p with its per-row 1/sum q): w = p * q,
    // rounded, i.e. exactly the materialised alpha
    float rs[CH];
#pragma unroll
    for (int ch = 0; ch < CH; ++ch) rs[ch] = (W && p.val_rs) ? p.val_rs[row * p.val_heads + cl.head[ch]] : 1.0f;
    for (int32_t j0 = 0; j0 < n; j0 += U) {
        int32_t c[U];
        V x[U][CH];
        float w[U][CH];
        float sc[U], sa[U];
        // one row per wave (G = 64): a batch's columns are wave-uniform, so one coalesced
        // load of U columns is spread to scalar registers (v_readlane) and the X row
        // addresses are formed on the scalar unit instead of per lane
        int32_t cu = 0;
        if constexpr (G == 64 && !SAMP) {
            const int kk = threadIdx.x & (U - 1);
            cu = p.col[e0 + ((j0 + kk < n) ? j0 + kk : n - 1)];
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int32_t jj = (j0 + k < n) ? j0 + k : n - 1;  // clamped: valid address
            const int32_t j = SAMP ? (p.ra * jj + p.rb) % deg : jj;
            const int64_t e = e0 + j;
            if constexpr (G == 64 && !SAMP)
                c[k] = __builtin_amdgcn_readlane(cu, k);
            else
                c[k] = p.col[e];
#pragma unroll
            for (int ch = 0; ch < CH; ++ch) w[k][ch] = W ? p.val[e * p.val_heads + cl.head[ch]] : 1.0f;
        }
        if (W && p.val_rs) {
#pragma unroll
            for (int k = 0; k < U; ++k)
#pragma unroll
                for (int ch = 0; ch < CH; ++ch) w[k][ch] = __fmul_rn(w[k][ch], rs[ch]);
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const float *xr = p.X + (int64_t)c[k] * p.ldx;
#pragma unroll
            for (int ch = 0; ch < CH; ++ch) x[k][ch] = ldv<VEC>(xr + cl.off[ch]);
            sc[k] = SRCS ? p.src_scale[c[k]] : 1.0f;
            sa[k] = (RELU && p.src_act) ? p.src_act[c[k]] : 1.0f;
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            if (j0 + k < n) {
#pragma unroll
                for (int ch = 0; ch < CH; ++ch)
                    accumulate<VEC, W, SRCS, RELU>(acc[ch], x[k][ch], w[k][ch], sc[k], sa[k]);
            }
        }
    }
}

// A column-tiled row (several segments, no sampling): the rowptr pairs of kSegGroup segments
// are loaded together and their edges walked as one list, segment order first, CSR order
// inside a segment (the per-segment loop's order, so the sums are bit-identical).  With
// col_tile(1000000) on an 11 M-row graph a row has ~0.2 edges per segment; the per-segment
// loop paid rowptr -> col -> X as three dependent misses per segment (12 segments: 11 ms
// per F = 128 call), here it is one of each per batch of U edges.
constexpr int kSegGroup = 8;
template <int VEC, int G, int CH, int U, bool W, bool SRCS, bool RELU = false>
__device__ __forceinline__ void accumulate_segments(const SpmmParams &p, KernargSegPtr seg, const Cols<VEC, G, CH, W> &cl,
                                                    int64_t row, typename VecT<VEC>::T (&acc)[CH]) {
    typedef typename VecT<VEC>::T V;
    const int64_t rp_stride = p.n_rows + 1;
    float rs[CH];
#pragma unroll
    for (int ch = 0; ch < CH; ++ch) rs[ch] = (W && p.val_rs) ? p.val_rs[row * p.val_heads + cl.head[ch]] : 1.0f;
    for (int s0 = 0; s0 < p.seg.n; s0 += kSegGroup) {
        int64_t lo[kSegGroup];
        int32_t pre[kSegGroup + 1];
        pre[0] = 0;
#pragma unroll
        for (int i = 0; i < kSegGroup; ++i) {
            const bool in = s0 + i < p.seg.n;
            const int s = in ? s0 + i : s0;
            const int32_t *rp = p.rowptr + (int64_t)seg->rp[s] * rp_stride;
            const int32_t a = rp[row], b = rp[row + 1];
            lo[i] = (int64_t)seg->base[s] + a;
            pre[i + 1] = pre[i] + (in ? b - a : 0);
        }
        const int32_t n = pre[kSegGroup];
        for (int32_t j0 = 0; j0 < n; j0 += U) {
            int32_t c[U];
            V x[U][CH];
            float w[U][CH];
            float sc[U], sa[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int32_t j = (j0 + k < n) ? j0 + k : n - 1;  // clamped: valid address
                // the last segment starting at or before j holds it (an empty one is passed)
                int64_t e = lo[0] + j;
#pragma unroll
                for (int i = 1; i < kSegGroup; ++i) e = (j >= pre[i]) ? lo[i] + (j - pre[i]) : e;
                c[k] = p.col[e];
#pragma unroll
                for (int ch = 0; ch < CH; ++ch) w[k][ch] = W ? p.val[e * p.val_heads + cl.head[ch]] : 1.0f;
            }
            if (W && p.val_rs) {
#pragma unroll
                for (int k = 0; k < U; ++k)
#pragma unroll
                    for (int ch = 0; ch < CH; ++ch) w[k][ch] = __fmul_rn(w[k][ch], rs[ch]);
            }
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const float *xr = p.X + (int64_t)c[k] * p.ldx;
#pragma unroll
                for (int ch = 0; ch < CH; ++ch) x[k][ch] = ldv<VEC>(xr + cl.off[ch]);
                sc[k] = SRCS ? p.src_scale[c[k]] : 1.0f;
                sa[k] = (RELU && p.src_act) ? p.src_act[c[k]] : 1.0f;
            }
#pragma unroll
            for (int k = 0; k < U; ++k) {
                if (j0 + k < n) {
#pragma unroll
                    for (int ch = 0; ch < CH; ++ch)
                        accumulate<VEC, W, SRCS, RELU>(acc[ch], x[k][ch], w[k][ch], sc[k], sa[k]);
                }
            }
        }
    }
}

template <int VEC, int G, int CH, bool W>
__device__ __forceinline__ void init_acc(const SpmmParams &p, const Cols<VEC, G, CH, W> &cl,
                                         int64_t row, typename VecT<VEC>::T (&acc)[CH]) {
    typedef typename VecT<VEC>::T V;
    const bool start_from_y = p.accum && p.dst_scale == nullptr && !p.dst_deg;
#pragma unroll
    for (int ch = 0; ch < CH; ++ch)
        acc[ch] = (start_from_y && cl.valid[ch]) ? ldv<VEC>(p.Y + row * p.ldy + cl.off[ch]) : V(0.0f);
}

template <int VEC, int G, int CH, bool W>
__device__ __forceinline__ void store_row(const SpmmParams &p, const Cols<VEC, G, CH, W> &cl,
                                          int64_t row, typename VecT<VEC>::T (&acc)[CH]) {
    typedef typename VecT<VEC>::T V;
    bool has_ds;
    const float ds = dst_factor(p, row, has_ds);
    const float s2 = p.y2_scale ? p.y2_scale[row] : ds;
#pragma unroll
    for (int ch = 0; ch < CH; ++ch) {
        if (!cl.valid[ch]) continue;
        float *yp = p.Y + row * p.ldy + cl.off[ch];
        V out = acc[ch];
        if (has_ds) {
#pragma unroll
            for (int i = 0; i < VEC; ++i) el<VEC>(out, i) = __fmul_rn(ds, el<VEC>(out, i));
            if (p.accum) {
                V y = ldv<VEC>(yp);
#pragma unroll
                for (int i = 0; i < VEC; ++i) el<VEC>(out, i) = __fadd_rn(el<VEC>(y, i), el<VEC>(out, i));
            }
        }
        if (p.relu_x) {  // the ReLU backward of the layer's input: gala_relu_scale_backward_f32's roundings
            const float a = p.relu_act ? p.relu_act[row] : 1.0f;
            V xv = ldv<VEC>(p.relu_x + row * p.ldrx + cl.off[ch]);
#pragma unroll
            for (int i = 0; i < VEC; ++i) {
                float t = el<VEC>(xv, i);
                if (p.relu_act) t = __fmul_rn(a, t);
                float d = relu_t(t) <= 0.0f ? 0.0f : el<VEC>(out, i);
                if (p.relu_act) d = __fmul_rn(d, a);
                el<VEC>(out, i) = d;
            }
        }
        stv_n<VEC>(yp, out, cl.nv[ch]);
        if (p.Y2) {  // the next aggregation's pre-scaled input, s2 * Y (its ROW_BROADCAST rounding)
#pragma unroll
            for (int i = 0; i < VEC; ++i) el<VEC>(out, i) = __fmul_rn(s2, el<VEC>(out, i));
            stv_n<VEC>(p.Y2 + row * p.ldy2 + cl.off[ch], out, cl.nv[ch]);
        }
    }
}

// the rows of row block `bid` of `nb` (skipping hub rows)
template <int VEC, int G, int CH, int U, bool W, bool SAMP, bool SRCS, bool RELU = false>
__device__ __forceinline__ void spmm_row_block(const SpmmParams &p, int64_t bid, int64_t nb) {
    typedef typename VecT<VEC>::T V;
    constexpr int RPW = kWave / G;
    const int lane = threadIdx.x & (kWave - 1);
    const int gl = lane & (G - 1);
    const int64_t blk = p.xcd_order ? logical_block_runs(bid, nb, kXcdRun) : bid;
    const int64_t wave = blk * (kBlock / kWave) + (threadIdx.x / kWave);
    const int64_t rid = wave * RPW + lane / G;
    if (rid >= p.n_rows) return;
    const int64_t row = p.row_order ? (int64_t)p.row_order[rid] : rid;
    KernargSegPtr seg = kernarg_segtable(offsetof(SpmmParams, seg));
    if (p.split_threshold > 0 && p.rowptr[row + 1] - p.rowptr[row] > p.split_threshold)
        return;  // hub row: its chunks (spmm_chunk_block) + k_spmm_fixup
    const Cols<VEC, G, CH, W> cl(p, gl);
    V acc[CH];
    init_acc<VEC, G, CH, W>(p, cl, row, acc);
    const int64_t rp_stride = p.n_rows + 1;
    const int nseg = p.seg.n;
    if (!SAMP && nseg > 1) {
        accumulate_segments<VEC, G, CH, U, W, SRCS, RELU>(p, seg, cl, row, acc);
        store_row<VEC, G, CH, W>(p, cl, row, acc);
        return;
    }
    for (int s = 0; s < nseg; ++s) {
        const int32_t *rp = p.rowptr + (int64_t)seg->rp[s] * rp_stride;
        const int64_t base = seg->base[s];
        accumulate_range<VEC, G, CH, U, W, SAMP, SRCS, RELU>(p, cl, row, base + rp[row], base + rp[row + 1], acc);
    }
    store_row<VEC, G, CH, W>(p, cl, row, acc);
}

template <int VEC, int G, int CH, int U, bool W, bool SAMP, bool SRCS, bool RELU = false>
__global__ __launch_bounds__(kBlock) void k_spmm_rowgroup(SpmmParams p) {
    spmm_row_block<VEC, G, CH, U, W, SAMP, SRCS, RELU>(p, blockIdx.x, gridDim.x);
}

// ---- split rows: chunk partials + ordered fix-up ---------------------------------------
struct SplitParams {
    const int32_t *rows;
    const int32_t *row_chunk0;
    const int32_t *chunk_row;
    float *ws;
    int64_t ws_cols;
    int64_t n_chunks;
    int64_t n_rows_split;
    int32_t chunk;
};

// the 512-edge chunks of hub rows in chunk block `bid` -> their partial sums in ws
template <int VEC, int G, int CH, int U, bool W, bool SRCS>
__device__ __forceinline__ void spmm_chunk_block(const SpmmParams &p, const SplitParams &sp, int64_t bid) {
    typedef typename VecT<VEC>::T V;
    constexpr int RPW = kWave / G;
    const int lane = threadIdx.x & (kWave - 1);
    const int gl = lane & (G - 1);
    const int64_t c = (bid * (kBlock / kWave) + threadIdx.x / kWave) * RPW + lane / G;
    if (c >= sp.n_chunks) return;
    const int32_t ri = sp.chunk_row[c];
    const int64_t row = sp.rows[ri];
    const int64_t k = c - sp.row_chunk0[ri];
    const int64_t r0 = p.rowptr[row], r1 = p.rowptr[row + 1];
    const int64_t e0 = r0 + k * sp.chunk;
    const int64_t e1 = (e0 + sp.chunk < r1) ? e0 + sp.chunk : r1;
    const Cols<VEC, G, CH, W> cl(p, gl);
    V acc[CH];
#pragma unroll
    for (int ch = 0; ch < CH; ++ch) acc[ch] = V(0.0f);
    accumulate_range<VEC, G, CH, U, W, false, SRCS>(p, cl, row, e0, e1, acc);
#pragma unroll
    for (int ch = 0; ch < CH; ++ch)
        if (cl.valid[ch]) stv<VEC>(sp.ws + c * sp.ws_cols + cl.off[ch], acc[ch]);
}

// A skewed graph's rows and hub-row chunks in ONE launch: the first `cb` blocks take the
// chunks (the largest, evenly sized pieces, dispatched first), the rest the row blocks in the
// plan's degree order.  One grid instead of two back to back: no drain / ramp between them.
template <int VEC, int G, int CH, int U, bool W, bool SRCS>
__global__ __launch_bounds__(kBlock) void k_spmm_rows_chunks(SpmmParams p, SplitParams sp, int64_t cb) {
    const int64_t b = blockIdx.x;
    if (b < cb)
        spmm_chunk_block<VEC, G, CH, U, W, SRCS>(p, sp, b);
    else
        spmm_row_block<VEC, G, CH, U, W, false, SRCS>(p, b - cb, (int64_t)gridDim.x - cb);
}

template <int VEC, int G, int CH, bool W>
__global__ __launch_bounds__(kBlock) void k_spmm_fixup(SpmmParams p, SplitParams sp) {
    typedef typename VecT<VEC>::T V;
    constexpr int RPW = kWave / G;
    constexpr int U = 8;
    const int lane = threadIdx.x & (kWave - 1);
    const int gl = lane & (G - 1);
    const int64_t ri = ((int64_t)blockIdx.x * (kBlock / kWave) + threadIdx.x / kWave) * RPW + lane / G;
    if (ri >= sp.n_rows_split) return;
    const int64_t row = sp.rows[ri];
    const Cols<VEC, G, CH, W> cl(p, gl);
    V acc[CH];
    init_acc<VEC, G, CH, W>(p, cl, row, acc);
    const int64_t c0 = sp.row_chunk0[ri], c1 = sp.row_chunk0[ri + 1];
    for (int64_t c = c0; c < c1; c += U) {
        V part[U][CH];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int64_t cc = (c + k < c1) ? c + k : c1 - 1;
#pragma unroll
            for (int ch = 0; ch < CH; ++ch) part[k][ch] = ldv<VEC>(sp.ws + cc * sp.ws_cols + cl.off[ch]);
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            if (c + k >= c1) continue;
#pragma unroll
            for (int ch = 0; ch < CH; ++ch)
#pragma unroll
                for (int i = 0; i < VEC; ++i)
                    el<VEC>(acc[ch], i) = __fadd_rn(el<VEC>(acc[ch], i), el<VEC>(part[k][ch], i));
        }
    }
    store_row<VEC, G, CH, W>(p, cl, row, acc);
}

// ---- hub rows in the reference's order ----------------------------------------------
// A hub row (deg > plan threshold) summed sequentially in CSR order, like every other row,
// so the result is bit-identical to the reference's serial row loop (cuda.h:286-358) --
// the REF parity mode.  One row group of G lanes would walk such a row one U-edge batch at
// a time, a dependent col -> X load chain per batch (a 388 K-edge R-MAT hub: ~100 ms).
// Instead one workgroup owns (row, slice of FSP features), split by role:
//   waves 1-7 (gatherers) fetch the X rows of tile t+1 (T edges, the next tiles' column
//        indices already loaded) and store them into one of two LDS buffers;
//   wave 0 (the chain) -- one lane per feature of the slice -- adds tile t from the other
//        buffer, in CSR order, with the per-feature operations and rounding of accumulate<>.
// One barrier per tile swaps the buffers, so the chain never waits for a gather or a store
// unless the gatherers fall behind.  Everything the chain reads is in LDS (X rows, src
// scales, edge weights, the accumulate start value): vmcnt counts in order, so one global
// load in the chain would wait for every gather issued before it.
constexpr int kHubThreads = 512;
constexpr int kHubGather = kHubThreads - kWave;  // gatherer lanes
constexpr int kHubBuf = 8192;      // floats of X per LDS buffer (32 KB; two buffers)
constexpr int kHubMaxHeads = 4;    // edge-weight heads per slice staged in LDS

struct HubParams {
    const int32_t *rows;           // hub row ids
    const int32_t *order;          // nullable: the plan's descending-degree row order
    int64_t n_hub;
    int32_t n_slices;              // ceil(F / FSP)
};

// LDS: buf[2][T/4][FSP][4] (X; an edge quad of one feature is one 16-B read; feature f in
// slot (f % VEC) * (FSP / VEC) + f / VEC of the quad's row), scl[2][T]
// (SRCS), wts[2][kHubMaxHeads][T] (W), yinit[64], then slack the chain's prefetch may read
// past a buffer (never consumed).  Unweighted: 68 KB, two workgroups per CU.
template <int FSP, bool W, bool SRCS>
struct HubLds {
    static constexpr int T = kHubBuf / FSP;          // edges per tile
    static constexpr int kGroup = 16;                 // edges per chain group
    static constexpr size_t buf = 0, scl = 2 * (size_t)kHubBuf, wts = scl + (SRCS ? 2 * T : 0),
                            yinit = wts + (W ? 2 * (size_t)kHubMaxHeads * T : 0), slack = yinit + kWave,
                            floats = slack + 2 * kGroup * FSP;
};

template <int VEC, int FSP, bool W, bool SRCS>
__global__ __launch_bounds__(kHubThreads) void k_spmm_hub_exact(SpmmParams p, HubParams hp) {
    typedef typename VecT<VEC>::T V;
    typedef HubLds<FSP, W, SRCS> L;
    constexpr int T = L::T;
    constexpr int RG = (T * (FSP / VEC) + kHubGather - 1) / kHubGather;  // loads per gatherer
    constexpr int RW = (T * kHubMaxHeads + kHubGather - 1) / kHubGather;
    extern __shared__ float hub_lds[];
    const int64_t ri = blockIdx.x / hp.n_slices;
    const int slice = blockIdx.x % hp.n_slices;
    // the plan's descending-degree row order starts with exactly the hub rows: the longest
    // serial chains are dispatched first
    const int64_t row = hp.order ? hp.order[ri] : hp.rows[ri];
    const int f0 = slice * FSP;
    const int fs = (p.F - f0) < FSP ? (p.F - f0) : FSP;  // features of the slice
    const int lpe = (fs + VEC - 1) / VEC;                // vectors per edge
    const int h0 = W ? f0 / p.head_dim : 0;               // edge-weight heads of the slice
    const int hs = W ? (f0 + fs - 1) / p.head_dim - h0 + 1 : 0;  // <= kHubMaxHeads (host)
    const int64_t e0 = p.rowptr[row], n = (int64_t)p.rowptr[row + 1] - e0;
    const int ntiles = (int)((n + T - 1) / T);
    const bool gatherer = threadIdx.x >= kWave;
    const int g = threadIdx.x - kWave;

    // ---- gatherers: slot k = (edge, column) of a tile, fixed for every tile ----
    int s_edge[RG], s_off[RG];
    int32_t cc[RG];
    V xr[RG];
    float sr[RG], wr[RW];
#pragma unroll
    for (int k = 0; k < RG; ++k) {
        const int i = k * kHubGather + g;
        s_edge[k] = (gatherer && i / lpe < T) ? i / lpe : -1;
        s_off[k] = (i % lpe) * VEC;
    }
    auto load_cols = [&](int t) {
#pragma unroll
        for (int k = 0; k < RG; ++k) {
            int64_t j = (int64_t)t * T + (s_edge[k] < 0 ? 0 : s_edge[k]);
            if (j >= n) j = n - 1;  // clamped: a valid address, never used
            cc[k] = p.col[e0 + j];
        }
    };
    auto load_x = [&](int t) {
        // unconditional (an unused slot's column is a valid one): branches around the
        // loads would make the compiler wait for each load before issuing the next
#pragma unroll
        for (int k = 0; k < RG; ++k) {
            xr[k] = ldv<VEC>(p.X + (int64_t)cc[k] * p.ldx + f0 + s_off[k]);
            if (SRCS) sr[k] = p.src_scale[cc[k]];
        }
        if (W) {  // weight (edge j, head h0 + k) for i = j * hs + k, coalesced along the edges
#pragma unroll
            for (int k = 0; k < RW; ++k) {
                const int i = k * kHubGather + g;
                int64_t j = (int64_t)t * T + (hs > 0 ? i / hs : 0);
                if (j >= n) j = n - 1;
                wr[k] = p.val[(e0 + j) * p.val_heads + h0 + (hs > 0 ? i % hs : 0)];
            }
        }
    };
    auto store = [&](int b) {
        float *xb = hub_lds + L::buf + (size_t)b * kHubBuf;
#pragma unroll
        for (int k = 0; k < RG; ++k) {
            const int e = s_edge[k];
            if (e < 0) continue;
            // feature f = s_off + v sits in slot v * (FSP / VEC) + s_off / VEC of its edge quad's
            // row (the chain lane of feature f reads that slot): the lanes of one store
            // instruction -- FSP / VEC features of 64 * VEC / FSP edges -- then fall on distinct
            // banks, where slot f put every fourth lane of a row on one bank (a 4-way conflict
            // on every gatherer store, stalling the chain's own LDS reads: the 388 K-edge R-MAT
            // chain 2.06 -> 1.80 ms, profiles/r06_hub_clock_swizzle.jsonl)
            float *q = xb + ((e >> 2) * FSP + s_off[k] / VEC) * 4 + (e & 3);
#pragma unroll
            for (int v = 0; v < VEC; ++v) q[4 * v * (FSP / VEC)] = el<VEC>(xr[k], v);
            if (SRCS && s_off[k] == 0) hub_lds[L::scl + b * T + e] = sr[k];
        }
        if (W) {
#pragma unroll
            for (int k = 0; k < RW; ++k) {
                const int i = k * kHubGather + g;
                if (i < T * hs) hub_lds[L::wts + (size_t)b * kHubMaxHeads * T + (i % hs) * T + i / hs] = wr[k];
            }
        }
    };

    // ---- chain: wave 0, lane f < fs owns feature f0 + f ----
    const int lane = threadIdx.x;
    const bool chain = lane < fs;
    const int cl = chain ? lane : 0;
    const int f = f0 + cl;
    const int slot = (cl % VEC) * (FSP / VEC) + cl / VEC;   // where the gatherers store feature cl
    const int hl = W ? f / p.head_dim - h0 : 0;
    const float rs = (W && p.val_rs) ? p.val_rs[row * p.val_heads + h0 + hl] : 1.0f;
    if (chain && p.accum && p.dst_scale == nullptr && !p.dst_deg) hub_lds[L::yinit + lane] = p.Y[row * p.ldy + f];
    float acc = 0.0f;
    auto add = [&](float x, float w, float sv) {
        const float v = SRCS ? __fmul_rn(sv, x) : x;
        if (W) acc = fmaf(p.val_rs ? __fmul_rn(w, rs) : w, v, acc);
        else acc = __fadd_rn(acc, v);
    };
    typedef float F4 __attribute__((ext_vector_type(4)));
    constexpr int GS = L::kGroup;
    struct Grp {
        F4 x[GS / 4], w[GS / 4], s[GS / 4];
    };
    auto run_chain = [&](int t) {
        const int b = t & 1;
        const float *xb = hub_lds + L::buf + (size_t)b * kHubBuf + slot * 4;
        const float *sb = hub_lds + L::scl + b * T;
        const float *wb = hub_lds + L::wts + (size_t)b * kHubMaxHeads * T + hl * T;
        const int cnt = (int)((n - (int64_t)t * T) < T ? (n - (int64_t)t * T) : T);
        auto fetch = [&](int j, Grp &q) {  // edges j .. j+GS-1 (j % 4 == 0): 16-B reads
#pragma unroll
            for (int u = 0; u < GS / 4; ++u) {
                q.x[u] = *reinterpret_cast<const F4 *>(xb + ((j >> 2) + u) * FSP * 4);
                if (SRCS) q.s[u] = *reinterpret_cast<const F4 *>(sb + j + 4 * u);
                if (W) q.w[u] = *reinterpret_cast<const F4 *>(wb + j + 4 * u);
            }
        };
        auto consume = [&](const Grp &q) {
#pragma unroll
            for (int u = 0; u < GS / 4; ++u)
#pragma unroll
                for (int v = 0; v < 4; ++v) add(q.x[u][v], W ? q.w[u][v] : 1.0f, SRCS ? q.s[u][v] : 1.0f);
        };
        // three groups in rotation: a group's 16-B reads are issued two groups ahead of its
        // adds (sched_barrier keeps that order; the scheduler would sink them to their use).
        // The prefetch past the last full round reads at most two groups past the buffer
        // (the other buffer or the slack) and is never consumed.
        int j = 0;
        const int full = cnt / (3 * GS) * (3 * GS);
        if (full > 0) {
            Grp A, B, C;
            fetch(0, A);
            fetch(GS, B);
            for (; j < full; j += 3 * GS) {
                fetch(j + 2 * GS, C);
                __builtin_amdgcn_sched_barrier(0);
                consume(A);
                __builtin_amdgcn_sched_barrier(0);
                fetch(j + 3 * GS, A);
                __builtin_amdgcn_sched_barrier(0);
                consume(B);
                __builtin_amdgcn_sched_barrier(0);
                fetch(j + 4 * GS, B);
                __builtin_amdgcn_sched_barrier(0);
                consume(C);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        for (; j + GS <= cnt; j += GS) {  // the remaining whole groups, one at a time
            Grp A;
            fetch(j, A);
            consume(A);
        }
        const float *xs = hub_lds + L::buf + (size_t)b * kHubBuf + slot * 4;
        for (; j < cnt; ++j)
            add(xs[(j >> 2) * FSP * 4 + (j & 3)], W ? wb[j] : 1.0f, SRCS ? sb[j] : 1.0f);
    };

    // ---- pipeline: tile t in buffer t&1 is added while tile t+1 is gathered into the other ----
    if (gatherer && ntiles > 0) {
        load_cols(0);
        load_x(0);
        if (ntiles > 1) load_cols(1);
        store(0);
        if (ntiles > 1) {
            load_x(1);
            if (ntiles > 2) load_cols(2);
        }
    }
    __syncthreads();
    if (chain && p.accum && p.dst_scale == nullptr && !p.dst_deg) acc = hub_lds[L::yinit + lane];
    for (int t = 0; t < ntiles; ++t) {
        if (gatherer) {
            if (t + 1 < ntiles) {
                store((t + 1) & 1);
                if (t + 2 < ntiles) {
                    load_x(t + 2);
                    if (t + 3 < ntiles) load_cols(t + 3);
                }
            }
        } else {
            run_chain(t);
        }
        __syncthreads();
    }
    if (!chain) return;
    float out = acc;
    bool has_ds;
    const float ds = dst_factor(p, row, has_ds);
    if (has_ds) {
        out = __fmul_rn(ds, out);
        if (p.accum) out = __fadd_rn(p.Y[row * p.ldy + f], out);
    }
    p.Y[row * p.ldy + f] = out;
    if (p.Y2) p.Y2[row * p.ldy2 + f] = __fmul_rn(p.y2_scale ? p.y2_scale[row] : ds, out);
}

// ---- degree: deg[r] = sum_e (val_e | 1), optionally ^power --------------------------
struct DegParams {
    const int32_t *rowptr;
    const float *val;
    float *deg;
    int64_t n_rows;
    float power;
    int32_t sample;
    int32_t nsamp;
    SegTable seg;
};

__global__ __launch_bounds__(kBlock) void k_degree_count(DegParams p) {
    const int64_t row = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (row >= p.n_rows) return;
    float d;
    if (p.sample) {
        d = (float)p.nsamp * (float)p.seg.n;  // FULL_OP: n * global_segments[0] (common.h:1358-1359)
    } else {
        int64_t cnt = 0;
        KernargSegPtr seg = kernarg_segtable(offsetof(DegParams, seg));
        for (int s = 0; s < p.seg.n; ++s) {
            const int32_t *rp = p.rowptr + (int64_t)seg->rp[s] * (p.n_rows + 1);
            cnt += rp[row + 1] - rp[row];
        }
        d = (float)cnt;  // exact: sequential sum of 1.0f is exact below 2^24
    }
    if (p.power != 1.0f) d = (p.power == -0.5f) ? deg_rsqrt(d) : powf(d, p.power);
    p.deg[row] = d;
}

// weighted degree: one row per 16-lane group, sequential per row to keep the order
__global__ __launch_bounds__(kBlock) void k_degree_weighted(DegParams p) {
    const int64_t row = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (row >= p.n_rows) return;
    float d = 0.0f;
    KernargSegPtr seg = kernarg_segtable(offsetof(DegParams, seg));
    for (int s = 0; s < p.seg.n; ++s) {
        const int32_t *rp = p.rowptr + (int64_t)seg->rp[s] * (p.n_rows + 1);
        const int64_t e0 = seg->base[s] + (int64_t)rp[row], e1 = seg->base[s] + (int64_t)rp[row + 1];
        for (int64_t e = e0; e < e1; ++e) d = __fadd_rn(d, p.val[e]);
    }
    if (p.power != 1.0f) d = (p.power == -0.5f) ? deg_rsqrt(d) : powf(d, p.power);
    p.deg[row] = d;
}

// ---- dispatch ---------------------------------------------------------------------------
template <int VEC, int G, int CH, int U, bool W, bool SAMP, bool SRCS, bool RELU = false>
static void launch_rg_u(const SpmmParams &p, const SplitParams *sp, hipStream_t st) {
    constexpr int rows_per_block = (kBlock / kWave) * (kWave / G);
    const int64_t blocks = (p.n_rows + rows_per_block - 1) / rows_per_block;
    if (RELU || SAMP || !sp || sp->n_chunks <= 0) {   // (the ReLU prologue: no hub split, host-checked)
        hipLaunchKernelGGL((k_spmm_rowgroup<VEC, G, CH, U, W, SAMP, SRCS, RELU>), dim3((unsigned)blocks),
                           dim3(kBlock), 0, st, p);
    }
    if constexpr (!RELU)
    if (!SAMP && sp && sp->n_chunks > 0) {
        const int64_t cb = (sp->n_chunks + rows_per_block - 1) / rows_per_block;
        hipLaunchKernelGGL((k_spmm_rows_chunks<VEC, G, CH, U, W, SRCS>), dim3((unsigned)(cb + blocks)),
                           dim3(kBlock), 0, st, p, *sp, cb);
        const int64_t fb = (sp->n_rows_split + rows_per_block - 1) / rows_per_block;
        hipLaunchKernelGGL((k_spmm_fixup<VEC, G, CH, W>), dim3((unsigned)fb), dim3(kBlock), 0, st, p,
                           *sp);
    }
}

template <int VEC, int FSP, bool W, bool SRCS>
static void launch_hub_t(const SpmmParams &p, HubParams hp, hipStream_t st) {
    constexpr size_t lds = HubLds<FSP, W, SRCS>::floats * sizeof(float);
    // more than the default 64 KB of dynamic LDS (gfx950 has 160 KB per CU): opt in once
    static const hipError_t opted = hipFuncSetAttribute((const void *)k_spmm_hub_exact<VEC, FSP, W, SRCS>,
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)opted;
    hp.n_slices = (p.F + FSP - 1) / FSP;
    hipLaunchKernelGGL((k_spmm_hub_exact<VEC, FSP, W, SRCS>), dim3((unsigned)(hp.n_hub * hp.n_slices)),
                       dim3(kHubThreads), lds, st, p, hp);
}

// slices of 32 features when F <= 32 (F = 32: one 128-B row per edge, 512 edges a tile),
// else of 64 (one chain lane per feature of a wave)
static void launch_hub(const SpmmParams &p, const HubParams &hp, int vec, bool w, bool srcs, hipStream_t st) {
#define GALA_HUB(V, S)                                                    \
    if (w) {                                                              \
        if (srcs) launch_hub_t<V, S, true, true>(p, hp, st);              \
        else launch_hub_t<V, S, true, false>(p, hp, st);                  \
    } else {                                                              \
        if (srcs) launch_hub_t<V, S, false, true>(p, hp, st);             \
        else launch_hub_t<V, S, false, false>(p, hp, st);                 \
    }
    const bool narrow = p.F <= 32;
    if (vec == 4) {
        if (narrow) { GALA_HUB(4, 32) } else { GALA_HUB(4, 64) }
    } else if (vec == 2) {
        if (narrow) { GALA_HUB(2, 32) } else { GALA_HUB(2, 64) }
    } else {
        if (narrow) { GALA_HUB(1, 32) } else { GALA_HUB(1, 64) }
    }
#undef GALA_HUB
}

template <int VEC, int G, int CH, bool W, bool SAMP, bool SRCS, bool RELU = false>
static void launch_rg(const SpmmParams &p, const SplitParams *sp, hipStream_t st) {
    // U: edges whose loads are in flight before the first add (per lane: U*CH vectors).
    // Measured on the Products shape (tools/spmm_sweep.py, uniform and R-MAT graphs):
    // 8 or 16 lanes per row (F = 32, 64) are fastest with 4 edges in flight (F = 32: 2.44
    // vs 2.60 ms at 8); narrower and wider rows keep 8.
    constexpr int U = (CH * VEC >= 16) ? 2 : (CH * VEC >= 8) ? 4 : (VEC == 4 && (G == 8 || G == 16)) ? 4 : 8;
    launch_rg_u<VEC, G, CH, U, W, SAMP, SRCS, RELU>(p, sp, st);
}

template <int VEC, int G, int CH>
static void launch_flags(const SpmmParams &p, const SplitParams *sp, bool w, bool samp, bool srcs,
                         hipStream_t st) {
    if (p.src_act || p.relu_prologue) {   // the ReLU prologue: unweighted, unsampled (host-checked)
        if (srcs) launch_rg<VEC, G, CH, false, false, true, true>(p, sp, st);
        else launch_rg<VEC, G, CH, false, false, false, true>(p, sp, st);
        return;
    }
    if (w) {
        if (samp) {
            if (srcs) launch_rg<VEC, G, CH, true, true, true>(p, sp, st);
            else launch_rg<VEC, G, CH, true, true, false>(p, sp, st);
        } else {
            if (srcs) launch_rg<VEC, G, CH, true, false, true>(p, sp, st);
            else launch_rg<VEC, G, CH, true, false, false>(p, sp, st);
        }
    } else {
        if (samp) {
            if (srcs) launch_rg<VEC, G, CH, false, true, true>(p, sp, st);
            else launch_rg<VEC, G, CH, false, true, false>(p, sp, st);
        } else {
            if (srcs) launch_rg<VEC, G, CH, false, false, true>(p, sp, st);
            else launch_rg<VEC, G, CH, false, false, false>(p, sp, st);
        }
    }
}

// Short rows (fewer than kSparseRowDeg edges on average: config 5's 11 M-row graph has
// 2.45) leave a row's U-edge batch mostly empty, and the kernel waits out rowptr -> col -> X
// once per row: its rate is rows in flight.  Rows of 5..64 float4 vectors then take half
// the lanes with two vectors each (G/2, CH = 2, U = 4: the same x registers per lane), i.e.
// twice the rows per wave.  The sums are unchanged (each lane still adds its features'
// edges in CSR order).  GALA_SPMM_SPARSE_ROWS=0 keeps the wide groups (measurement).
constexpr int64_t kSparseRowDeg = 8;
static bool sparse_rows_enabled() {
    static const bool on = [] {
        const char *v = std::getenv("GALA_SPMM_SPARSE_ROWS");
        return !(v && v[0] == '0');
    }();
    return on;
}

template <int VEC>
static int launch_vec(const SpmmParams &p, const SplitParams *sp, int L, bool w, bool samp,
                      bool srcs, hipStream_t st, bool sparse_rows = false) {
    if (VEC == 4 && sparse_rows && L > 4 && L <= 64) {
        if (L <= 8) launch_flags<VEC, 4, 2>(p, sp, w, samp, srcs, st);
        else if (L <= 16) launch_flags<VEC, 8, 2>(p, sp, w, samp, srcs, st);
        else if (L <= 32) launch_flags<VEC, 16, 2>(p, sp, w, samp, srcs, st);
        else launch_flags<VEC, 32, 2>(p, sp, w, samp, srcs, st);
        return GALA_OK;
    }
    // L = vector elements per row (ceil(F/VEC)).  Rows that are not a multiple of 4 floats
    // (VEC < 4) and span 17..64 vectors (F = 47, the Products class count) take 16 lanes
    // with ceil(L/16) chunks each rather than 64 lanes with one: 4 rows per wave.
    if (VEC < 4 && L > 16 && L <= 64) {
        const int ch = (L + 15) / 16;
        if (ch == 2) launch_flags<VEC, 16, 2>(p, sp, w, samp, srcs, st);
        else if (ch == 3) launch_flags<VEC, 16, 3>(p, sp, w, samp, srcs, st);
        else launch_flags<VEC, 16, 4>(p, sp, w, samp, srcs, st);
        return GALA_OK;
    }
    if (L <= 1) launch_flags<VEC, 1, 1>(p, sp, w, samp, srcs, st);
    else if (L <= 2) launch_flags<VEC, 2, 1>(p, sp, w, samp, srcs, st);
    else if (L <= 4) launch_flags<VEC, 4, 1>(p, sp, w, samp, srcs, st);
    else if (L <= 8) launch_flags<VEC, 8, 1>(p, sp, w, samp, srcs, st);
    else if (L <= 16) launch_flags<VEC, 16, 1>(p, sp, w, samp, srcs, st);
    else if (L <= 32) launch_flags<VEC, 32, 1>(p, sp, w, samp, srcs, st);
    else if (L <= 64) launch_flags<VEC, 64, 1>(p, sp, w, samp, srcs, st);
    else if (L <= 128) launch_flags<VEC, 64, 2>(p, sp, w, samp, srcs, st);
    else if (L <= 192) launch_flags<VEC, 64, 3>(p, sp, w, samp, srcs, st);
    else if (L <= 256) launch_flags<VEC, 64, 4>(p, sp, w, samp, srcs, st);
    else if (L <= 384) launch_flags<VEC, 64, 6>(p, sp, w, samp, srcs, st);
    else if (L <= 512) launch_flags<VEC, 64, 8>(p, sp, w, samp, srcs, st);
    else return GALA_ERR_UNSUPPORTED;
    return GALA_OK;
}

}  // namespace gala

using namespace gala;

extern "C" int gala_spmm_f32(const gala_csr_t *A, const float *X, int64_t ldx, float *Y,
                             int64_t ldy, int32_t F, const float *src_scale,
                             const float *dst_scale, int32_t flags, int32_t nsamp, int32_t ra,
                             int32_t rb, void *stream) {
    return gala_spmm_ex_f32(A, X, ldx, Y, ldy, F, src_scale, dst_scale, flags, nsamp, ra, rb, nullptr, stream);
}

extern "C" int gala_spmm_ex_f32(const gala_csr_t *A, const float *X, int64_t ldx, float *Y,
                                int64_t ldy, int32_t F, const float *src_scale,
                                const float *dst_scale, int32_t flags, int32_t nsamp, int32_t ra,
                                int32_t rb, const gala_spmm_epilogue_t *epi, void *stream) {
    int st = check_csr(A);
    if (st) return st;
    const bool dst_deg = epi && epi->dst_deg_rsqrt;
    float *Y2 = epi ? epi->Y2 : nullptr;
    const int64_t ldy2 = Y2 ? epi->ldy2 : 0;
    const bool relu_pro = epi && epi->src_relu;
    const float *relu_x = epi ? epi->relu_x : nullptr;
    const int64_t ldrx = relu_x ? epi->ldrx : 0;
    if (epi && epi->src_act && !relu_pro) return GALA_ERR_INVALID_ARG;
    if (relu_x && ldrx < F) return GALA_ERR_INVALID_ARG;
    if ((relu_pro || relu_x) &&
        (A->val || (flags & GALA_SPMM_SAMPLE) || Y2 || (A->split && A->split->n_rows_split > 0)))
        return GALA_ERR_UNSUPPORTED;
    // the deg norm is the unweighted degree (rowptr counts): refused on weighted graphs, whose
    // degree pass sums the values (k_degree_weighted)
    if (dst_deg && (dst_scale || A->n_seg != 1 || A->val || (flags & GALA_SPMM_SAMPLE))) return GALA_ERR_UNSUPPORTED;
    if (Y2 && ldy2 < F) return GALA_ERR_INVALID_ARG;
    if (F < 0 || ldx < F || ldy < F ||
        (flags & ~(GALA_SPMM_ACCUM | GALA_SPMM_SAMPLE | GALA_SPMM_EXACT | GALA_SPMM_HUB_CHUNKED)) ||
        ((flags & GALA_SPMM_EXACT) && (flags & GALA_SPMM_HUB_CHUNKED)))
        return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0 || F == 0) return GALA_OK;
    if (!Y || (!X && A->nnz > 0)) return GALA_ERR_INVALID_ARG;
    const bool samp = (flags & GALA_SPMM_SAMPLE) != 0;
    if (samp && nsamp < 0) return GALA_ERR_INVALID_ARG;
    const bool w = A->val != nullptr;
    if (w && (A->val_heads < 1 || F % A->val_heads != 0)) return GALA_ERR_INVALID_ARG;
    if (A->val_row_scale && !w) return GALA_ERR_INVALID_ARG;
    const int32_t head_dim = w ? F / A->val_heads : F;

    // widest vector that divides both strides with aligned bases and either divides F and
    // the head width, or fits padded rows (one head, ldx and ldy >= F rounded up to it:
    // the padding is read, never written)
    // (a hub-row workspace row then holds whole vectors: ws_cols a multiple of VEC and at
    // least the padded width)
    int vec = 4;
    const bool one_head = !w || A->val_heads == 1;
    const gala_split_plan_t *plan = A->split;
    // hub rows: by default (REF order) summed sequentially by k_spmm_hub_exact; with
    // GALA_SPMM_HUB_CHUNKED as chunk partials + an ordered fix-up (the fast, reordered mode)
    const bool has_hubs = plan && plan->n_rows_split > 0 && A->n_seg == 1 && !samp;
    const bool use_split = has_hubs && plan->n_chunks > 0 && (flags & GALA_SPMM_HUB_CHUNKED);
    // the hub kernel stages at most kHubMaxHeads edge-weight heads per feature slice in LDS;
    // narrower heads keep the hub rows in the row kernel (one sequential pass: exact, slow)
    bool heads_ok = true;
    if (A->val && A->val_heads > 1) {
        const int hd = F / A->val_heads, fsp = F <= 32 ? 32 : 64;
        for (int f0 = 0; f0 < F && hd > 0; f0 += fsp) {
            const int f1 = (f0 + fsp < F ? f0 + fsp : F) - 1;
            if (f1 / hd - f0 / hd + 1 > kHubMaxHeads) heads_ok = false;
        }
    }
    const bool use_hub = has_hubs && !use_split && heads_ok;
    auto ok = [&](int v) {
        const int64_t Fv = ((int64_t)F + v - 1) / v * v;
        const bool fits = (F % v == 0 && head_dim % v == 0) || (one_head && ldx >= Fv && ldy >= Fv);
        const int64_t wcols = Fv < 512LL * v ? Fv : 512LL * v;
        const bool ws_ok = !use_split || (plan->ws_cols % v == 0 && plan->ws_cols >= wcols);
        const bool y2_ok = !Y2 || (ldy2 % v == 0 && ((uintptr_t)Y2 % (4 * v)) == 0 && (F % v == 0 || ldy2 >= Fv));
        const bool rx_ok = !relu_x || (ldrx % v == 0 && ((uintptr_t)relu_x % (4 * v)) == 0 && (F % v == 0 || ldrx >= Fv));
        return fits && ws_ok && y2_ok && rx_ok && ldx % v == 0 && ldy % v == 0 && ((uintptr_t)X % (4 * v)) == 0 &&
               ((uintptr_t)Y % (4 * v)) == 0;
    };
    while (vec > 1 && !ok(vec)) vec >>= 1;

    SpmmParams p;
    p.rowptr = A->rowptr;
    p.col = A->col;
    p.val = A->val;
    p.val_rs = A->val_row_scale;
    p.X = X;
    p.Y = Y;
    p.src_scale = src_scale;
    p.dst_scale = dst_scale;
    p.n_rows = A->n_rows;
    p.ldx = ldx;
    p.ldy = ldy;
    p.F = F;
    p.val_heads = w ? A->val_heads : 1;
    p.head_dim = head_dim;
    p.nsamp = nsamp;
    p.ra = ra;
    p.rb = rb;
    p.split_threshold = 0;
    p.dst_deg = dst_deg ? 1 : 0;
    p.Y2 = Y2;
    p.ldy2 = ldy2;
    p.y2_scale = Y2 ? epi->y2_scale : nullptr;
    p.relu_prologue = relu_pro ? 1 : 0;
    p.src_act = relu_pro ? epi->src_act : nullptr;
    p.relu_x = relu_x;
    p.ldrx = ldrx;
    p.relu_act = relu_x ? epi->relu_act : nullptr;
    p.row_order = nullptr;
    p.xcd_order = 1;  // off below when a degree-ordered row schedule is used (heavy rows first)
    hipStream_t hs = (hipStream_t)stream;

    // hub rows: chunk partials + ordered fix-up (plan built once per graph on the host)
    SplitParams spl{};
    const SplitParams *sp = nullptr;
    if (plan && plan->row_order && A->n_seg == 1) {
        p.row_order = plan->row_order;
        p.xcd_order = 0;
    }
    if (use_split) {
        if (plan->threshold < 1 || plan->chunk < 1 || !plan->rows || !plan->row_chunk0 ||
            !plan->chunk_row || !plan->workspace)
            return GALA_ERR_INVALID_ARG;
        spl.rows = plan->rows;
        spl.row_chunk0 = plan->row_chunk0;
        spl.chunk_row = plan->chunk_row;
        spl.ws = plan->workspace;
        spl.ws_cols = plan->ws_cols;
        spl.n_chunks = plan->n_chunks;
        spl.n_rows_split = plan->n_rows_split;
        spl.chunk = plan->chunk;
        p.split_threshold = plan->threshold;
        sp = &spl;
    }
    HubParams hp{};
    hipStream_t hub_st = hs;
    if (use_hub) {
        if (plan->threshold < 1 || !plan->rows) return GALA_ERR_INVALID_ARG;
        p.split_threshold = plan->threshold;  // the row kernel leaves hub rows to k_spmm_hub_exact
        hp.rows = plan->rows;
        hp.order = plan->row_order;
        hp.n_hub = plan->n_rows_split;
        // the hub rows run beside the row kernel on the plan's side stream when it has one
        if (plan->aux_stream && plan->aux_events[0] && plan->aux_events[1]) hub_st = (hipStream_t)plan->aux_stream;
    }

    // feature chunks wider than 512 vectors per lane-group are split over launches
    const int64_t max_cols = 512LL * vec;
    if (sp && plan->ws_cols < (F < max_cols ? F : max_cols)) return GALA_ERR_INVALID_ARG;
    if (w && p.val_heads > 1 && F > max_cols) return GALA_ERR_UNSUPPORTED;
    for (int32_t seg0 = 0; seg0 < A->n_seg; seg0 += kMaxSegPerLaunch) {
        st = fill_segments(A, seg0, &p.seg);
        if (st) return st;
        // segments after the first launch always accumulate onto the previous ones
        const bool accum = (flags & GALA_SPMM_ACCUM) || seg0 > 0;
        if (seg0 > 0 && (dst_scale || Y2)) return GALA_ERR_UNSUPPORTED;
        for (int64_t c0 = 0; c0 < F; c0 += max_cols) {
            const int32_t Fc = (int32_t)((F - c0) < max_cols ? (F - c0) : max_cols);
            SpmmParams q = p;
            q.X = X ? X + c0 : nullptr;
            q.Y = Y + c0;
            q.Y2 = Y2 ? Y2 + c0 : nullptr;
            // the ReLU backward belongs to the finished row: only the launch of the last segment
            // group applies it (earlier launches leave the partial sums for it to accumulate)
            q.relu_x = relu_x && seg0 + kMaxSegPerLaunch >= A->n_seg ? relu_x + c0 : nullptr;
            if (!q.relu_x) q.relu_act = nullptr;
            q.F = Fc;
            q.accum = accum;
            const int L = (int)((Fc + vec - 1) / vec);
            int r = 0;
            const bool forked = use_hub && hub_st != hs;
            if (use_hub) {  // the long serial rows first, so their workgroups are dispatched first
                if (forked) {
                    if (hipEventRecord((hipEvent_t)plan->aux_events[0], hs) != hipSuccess ||
                        hipStreamWaitEvent(hub_st, (hipEvent_t)plan->aux_events[0], 0) != hipSuccess)
                        return launch_status();
                }
                launch_hub(q, hp, vec, w, src_scale != nullptr, hub_st);
                r = launch_status();
            }
            if (!r) {
                const bool sparse_rows =
                    sparse_rows_enabled() && A->n_rows > 0 && A->nnz < kSparseRowDeg * (int64_t)A->n_rows;
                if (vec == 4) r = launch_vec<4>(q, sp, L, w, samp, src_scale != nullptr, hs, sparse_rows);
                else if (vec == 2) r = launch_vec<2>(q, sp, L, w, samp, src_scale != nullptr, hs);
                else r = launch_vec<1>(q, sp, L, w, samp, src_scale != nullptr, hs);
                if (!r) r = launch_status();
            }
            // join (also after a failed launch, so a fork never stays open -- an unjoined fork
            // would invalidate a hipGraph capture on the caller's stream): the caller's stream
            // waits for the hub rows
            if (forked) {
                if (hipEventRecord((hipEvent_t)plan->aux_events[1], hub_st) != hipSuccess ||
                    hipStreamWaitEvent(hs, (hipEvent_t)plan->aux_events[1], 0) != hipSuccess) {
                    const int j = launch_status();
                    if (!r) r = j ? j : GALA_ERR_HIP;
                }
            }
            if (r) return r;
        }
    }
    return GALA_OK;
}

extern "C" int gala_degree_f32(const gala_csr_t *A, float *deg, float power, int32_t flags,
                               int32_t nsamp, void *stream) {
    int st = check_csr(A);
    if (st) return st;
    if (!deg || (flags & ~(GALA_SPMM_SAMPLE))) return GALA_ERR_INVALID_ARG;
    if (A->n_rows == 0) return GALA_OK;
    if (A->n_seg > kMaxSegPerLaunch) return GALA_ERR_UNSUPPORTED;
    DegParams p;
    p.rowptr = A->rowptr;
    p.val = A->val;
    p.deg = deg;
    p.n_rows = A->n_rows;
    p.power = power;
    p.sample = (flags & GALA_SPMM_SAMPLE) ? 1 : 0;
    p.nsamp = nsamp;
    st = fill_segments(A, 0, &p.seg);
    if (st) return st;
    const int64_t blocks = (A->n_rows + kBlock - 1) / kBlock;
    if (A->val && !p.sample)
        hipLaunchKernelGGL(k_degree_weighted, dim3((unsigned)blocks), dim3(kBlock), 0,
                           (hipStream_t)stream, p);
    else
        hipLaunchKernelGGL(k_degree_count, dim3((unsigned)blocks), dim3(kBlock), 0,
                           (hipStream_t)stream, p);
    return launch_status();
}

namespace gala {

// ---- row-wise elementwise ops (ROW_BROADCAST and the GCN ReLU prologue) ----------------
// Grid-stride over (row, vector) pairs with the row / column stepped incrementally (no
// per-element 64-bit division).  A padded row's last vector (F % VEC != 0, strides padded
// to VEC; checked on the host) computes on its padding and stores only the real columns.
template <int VEC>
__device__ __forceinline__ void store_cols(float *p, const typename VecT<VEC>::T &v, int nv) {
    stv_n<VEC>(p, v, nv);
}

// ROW_BROADCAST: Y[r,:] = scale[r] * X[r,:]
struct RowBroadcastOp {
    const float *scale, *X;
    float *Y;
    int64_t ldx, ldy;
    template <int VEC>
    __device__ __forceinline__ void apply(int64_t r, int64_t c, int nv) const {
        const float s = scale[r];
        typename VecT<VEC>::T v = ldv<VEC>(X + r * ldx + c);
#pragma unroll
        for (int i = 0; i < VEC; ++i) el<VEC>(v, i) = __fmul_rn(s, el<VEC>(v, i));
        store_cols<VEC>(Y + r * ldy + c, v, nv);
    }
};

// torch.relu as its GPU kernel computes it: t > 0 ? t : +0, NaN passes through


// Y[r,:] = pre[r] * relu(act[r] * X[r,:]), each factor optional (absent: no rounding step)
struct ScaleReluOp {
    const float *act, *pre, *X;
    float *Y;
    int64_t ldx, ldy;
    template <int VEC>
    __device__ __forceinline__ void apply(int64_t r, int64_t c, int nv) const {
        const float a = act ? act[r] : 1.0f, b = pre ? pre[r] : 1.0f;
        typename VecT<VEC>::T v = ldv<VEC>(X + r * ldx + c);
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
            float t = el<VEC>(v, i);
            if (act) t = __fmul_rn(a, t);
            t = relu_t(t);
            if (pre) t = __fmul_rn(b, t);
            el<VEC>(v, i) = t;
        }
        store_cols<VEC>(Y + r * ldy + c, v, nv);
    }
};

// its backward: dX[r,:] = act[r] * (act[r] * X[r,:] <= 0 ? 0 : G[r,:])
// (threshold_backward on the ReLU output, then the product rule of act * X)
struct ReluScaleBwdOp {
    const float *act, *X, *G;
    float *dX;
    int64_t ldx, ldg, lddx;
    template <int VEC>
    __device__ __forceinline__ void apply(int64_t r, int64_t c, int nv) const {
        const float a = act ? act[r] : 1.0f;
        typename VecT<VEC>::T v = ldv<VEC>(X + r * ldx + c);
        const typename VecT<VEC>::T g = ldv<VEC>(G + r * ldg + c);
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
            float t = el<VEC>(v, i);
            if (act) t = __fmul_rn(a, t);
            float d = relu_t(t) <= 0.0f ? 0.0f : reinterpret_cast<const float *>(&g)[i];
            if (act) d = __fmul_rn(d, a);
            el<VEC>(v, i) = d;
        }
        store_cols<VEC>(dX + r * lddx + c, v, nv);
    }
};

template <int VEC, class Op>
__global__ __launch_bounds__(kBlock) void k_rows(int64_t n_rows, int32_t F, int32_t L, Op op) {
    const int64_t t0 = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    int64_t r = t0 / L, c = t0 % L;
    const int64_t dr = stride / L, dc = stride % L;
    while (r < n_rows) {
        const int64_t col = c * VEC;
        op.template apply<VEC>(r, col, F - col < VEC ? (int)(F - col) : VEC);
        c += dc;
        r += dr;
        if (c >= L) {
            c -= L;
            ++r;
        }
    }
}

// widest vector for row ops over [n_rows, F] with the given strides / bases: VEC divides F,
// or the rows are padded to it (every stride >= F rounded up to VEC)
static int rows_vec(int32_t F, std::initializer_list<int64_t> lds, std::initializer_list<const void *> ptrs) {
    for (int v = 4; v > 1; v >>= 1) {
        const int64_t Fv = ((int64_t)F + v - 1) / v * v;
        bool ok = true;
        for (int64_t ld : lds) ok = ok && ld % v == 0 && (F % v == 0 || ld >= Fv);
        for (const void *q : ptrs) ok = ok && ((uintptr_t)q % (4 * v)) == 0;
        if (ok) return v;
    }
    return 1;
}

template <class Op>
static int launch_rows(int64_t n_rows, int32_t F, int vec, const Op &op, void *stream) {
    const int32_t L = (F + vec - 1) / vec;
    const int64_t total = n_rows * L;
    int64_t blocks = (total + kBlock - 1) / kBlock;
    if (blocks > 256 * 16) blocks = 256 * 16;  // grid-stride: 16 workgroups per CU
    hipStream_t hs = (hipStream_t)stream;
    if (vec == 4) hipLaunchKernelGGL((k_rows<4, Op>), dim3((unsigned)blocks), dim3(kBlock), 0, hs, n_rows, F, L, op);
    else if (vec == 2) hipLaunchKernelGGL((k_rows<2, Op>), dim3((unsigned)blocks), dim3(kBlock), 0, hs, n_rows, F, L, op);
    else hipLaunchKernelGGL((k_rows<1, Op>), dim3((unsigned)blocks), dim3(kBlock), 0, hs, n_rows, F, L, op);
    return launch_status();
}

}  // namespace gala

extern "C" int gala_row_broadcast_f32(int64_t n_rows, int32_t F, const float *scale,
                                      const float *X, int64_t ldx, float *Y, int64_t ldy,
                                      void *stream) {
    if (n_rows < 0 || F < 0 || ldx < F || ldy < F) return GALA_ERR_INVALID_ARG;
    if (n_rows == 0 || F == 0) return GALA_OK;
    if (!scale || !X || !Y) return GALA_ERR_INVALID_ARG;
    return gala::launch_rows(n_rows, F, gala::rows_vec(F, {ldx, ldy}, {X, Y}),
                             gala::RowBroadcastOp{scale, X, Y, ldx, ldy}, stream);
}

namespace gala {
// ROW_BROADCAST of the GCN norm computed from the graph: Y[r,:] = deg(r)^-0.5 * X[r,:]
// (one segment), the degree pass and the `norm * res` product in one elementwise pass
struct DegBroadcastOp {
    const int32_t *rowptr;
    const float *X;
    float *Y;
    int64_t ldx, ldy;
    template <int VEC>
    __device__ __forceinline__ void apply(int64_t r, int64_t c, int nv) const {
        const float s = deg_rsqrt((float)(rowptr[r + 1] - rowptr[r]));
        typename VecT<VEC>::T v = ldv<VEC>(X + r * ldx + c);
#pragma unroll
        for (int i = 0; i < VEC; ++i) el<VEC>(v, i) = __fmul_rn(s, el<VEC>(v, i));
        store_cols<VEC>(Y + r * ldy + c, v, nv);
    }
};
}  // namespace gala

extern "C" int gala_row_broadcast_deg_f32(const gala_csr_t *A, int32_t F, const float *X, int64_t ldx,
                                          float *Y, int64_t ldy, void *stream) {
    int st = check_csr(A);
    if (st) return st;
    if (F < 0 || ldx < F || ldy < F) return GALA_ERR_INVALID_ARG;
    if (A->n_seg != 1 || A->val) return GALA_ERR_UNSUPPORTED;  // rowptr counts: unweighted degree only
    if (A->n_rows == 0 || F == 0) return GALA_OK;
    if (!X || !Y) return GALA_ERR_INVALID_ARG;
    return gala::launch_rows(A->n_rows, F, gala::rows_vec(F, {ldx, ldy}, {X, Y}),
                             gala::DegBroadcastOp{A->rowptr, X, Y, ldx, ldy}, stream);
}

extern "C" int gala_row_scale_relu_f32(int64_t n_rows, int32_t F, const float *act,
                                       const float *pre, const float *X, int64_t ldx, float *Y,
                                       int64_t ldy, void *stream) {
    if (n_rows < 0 || F < 0 || ldx < F || ldy < F) return GALA_ERR_INVALID_ARG;
    if (n_rows == 0 || F == 0) return GALA_OK;
    if (!X || !Y) return GALA_ERR_INVALID_ARG;
    return gala::launch_rows(n_rows, F, gala::rows_vec(F, {ldx, ldy}, {X, Y}),
                             gala::ScaleReluOp{act, pre, X, Y, ldx, ldy}, stream);
}

extern "C" int gala_relu_scale_backward_f32(int64_t n_rows, int32_t F, const float *act,
                                            const float *X, int64_t ldx, const float *G,
                                            int64_t ldg, float *dX, int64_t lddx, void *stream) {
    if (n_rows < 0 || F < 0 || ldx < F || ldg < F || lddx < F) return GALA_ERR_INVALID_ARG;
    if (n_rows == 0 || F == 0) return GALA_OK;
    if (!X || !G || !dX) return GALA_ERR_INVALID_ARG;
    return gala::launch_rows(n_rows, F, gala::rows_vec(F, {ldx, ldg, lddx}, {X, G, dX}),
                             gala::ReluScaleBwdOp{act, X, G, dX, ldx, ldg, lddx}, stream);
}

