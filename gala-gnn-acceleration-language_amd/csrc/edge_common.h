// edge_common.h -- shared by the edge-op kernels (edge.hip) and the fused GAT kernels
// (gat.hip): the kernel argument block, row / chunk prologues, hub-row split, register
// tiles, per-lane feature ownership with row padding, and the host-side launch helpers.
#pragma once

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

// Register tiles: a row slice is walked in tiles of G*K values; lane g holds the values
// t0 + g + k*G (k < K), so every lane has K coalesced loads in flight before it uses any
// (one load per lane at a time left these kernels latency-bound: 0.5 TB/s at 8 heads).
// When a row fits one tile, the second pass of softmax fwd/bwd runs from the registers.
constexpr int kTileK = 8;

// over the lanes of one head: partners G/2, ..., HP (lane_xor: DPP below 16)
template <int G, int HP>
__device__ __forceinline__ float head_sum(float v) {
    if constexpr (G / 2 >= HP && G >= 2) {
        v += lane_xor<G / 2>(v);
        return head_sum<G / 2, HP>(v);
    } else {
        return v;
    }
}
template <int G, int HP>
__device__ __forceinline__ float head_max(float v) {
    if constexpr (G / 2 >= HP && G >= 2) {
        v = fmaxf(v, lane_xor<G / 2>(v));
        return head_max<G / 2, HP>(v);
    } else {
        return v;
    }
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

__device__ __forceinline__ float ref_exp(float s) {
    // torch::exp then torch::clamp(0, 1e12) (common.h:760-761); NaN propagates like clamp
    const float p = expf(s);
    return p > 1e12f ? 1e12f : p;
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

// ---- host side ------------------------------------------------------------------------
static inline int pick_group(const gala_csr_t *A, int heads) {
    // lanes per row from the mean row length (edges*heads)
    // ~2-4 edges per lane: several rows per wave amortise the per-row bookkeeping
    const double avg = A->n_rows ? (double)A->nnz * heads / (double)A->n_rows : 1.0;
    int g = 4;
    while (g < 64 && 2 * g * 2 <= avg) g <<= 1;
    return g;
}

// lanes per row for the register-tiled kernels: the smallest group whose tile (G*K
// values) holds a mean row with 15 % slack, so most rows take one tile
static inline int pick_group_tiled(const gala_csr_t *A, int heads) {
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
static inline int64_t pad_to(int64_t F, int v) { return (F + v - 1) / v * v; }

static inline int narrow_chunks(int heads, int vec, int L) {
    return (heads == 1 && vec < 4 && L > 16 && L <= 64) ? (L + 15) / 16 : 1;
}

static inline int edge_setup(const gala_csr_t *A, int32_t heads, EdgeParams *p) {
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

static inline unsigned blocks_for(int64_t n_rows, int G) {
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
static inline int pow2_heads(int heads) {
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

static inline unsigned blocks_for_groups(int64_t n, int G) {
    const int64_t per_block = (int64_t)(kBlock / kWave) * (kWave / G);
    return (unsigned)((n + per_block - 1) / per_block);
}

// the hub-row plan of A, when it applies and its workspace holds `need` floats per chunk
// (otherwise hub rows run in one pass, like every other row)
static inline bool hub_split(const gala_csr_t *A, int64_t need, HubSplit *sp) {
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

// REF-order hub kernels run beside the row kernel on the plan's side stream when it has one
// (gala_split_plan_t.aux_stream / aux_events): fork() makes the side stream wait for the
// caller's, join(status) makes the caller's wait for the side stream -- also after a failed
// launch, so a fork never stays open (that would invalidate a hipGraph capture).  Without
// a side stream both are no-ops and `side` is the caller's stream.
struct HubFork {
    hipStream_t main, side;
    hipEvent_t ev[2];
    bool forked = false;
    HubFork(const gala_split_plan_t *plan, hipStream_t hs) : main(hs), side(hs) {
        if (plan && plan->aux_stream && plan->aux_events[0] && plan->aux_events[1]) {
            side = (hipStream_t)plan->aux_stream;
            ev[0] = (hipEvent_t)plan->aux_events[0];
            ev[1] = (hipEvent_t)plan->aux_events[1];
        }
    }
    int fork() {
        if (side == main) return GALA_OK;
        if (hipEventRecord(ev[0], main) != hipSuccess || hipStreamWaitEvent(side, ev[0], 0) != hipSuccess)
            return launch_status();
        forked = true;
        return GALA_OK;
    }
    int join(int st) {
        if (!forked) return st;
        forked = false;
        if (hipEventRecord(ev[1], side) != hipSuccess || hipStreamWaitEvent(main, ev[1], 0) != hipSuccess) {
            const int j = launch_status();
            return st ? st : (j ? j : GALA_ERR_HIP);
        }
        return st;
    }
};

}  // namespace gala
