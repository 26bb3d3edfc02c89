// dense.hip — weight / bias gradients of the FFN (FFN_OP) for tall-skinny node matrices.
//
// The generated programs' FFNs are torch Linear layers on [N, K] node features with
// N = 10^5..10^8 and K, M <= a few hundred (gala.cu:415-420, common.h:1188-1242).  Their
// backward needs dW[m, k] = sum_n dY[n, m] X[n, k] and db[m] = sum_n dY[n, m]: a GEMM whose
// contraction runs over the N rows.  Measured on the Products GCN program, torch's bias
// reduction over dim 0 takes 18.6 ms and the weight GEMM 3.3 ms (profiles/r01_e2e_*), for
// 1.3 GB of input that HBM streams in ~0.2 ms.  Here the rows are split into P chunks
// (split-K): every workgroup accumulates one (m, k) tile (64x64, or 32x128 for narrow M)
// of one chunk in registers (4x4 per lane, both operands staged through LDS 32 rows at a
// time, the next step prefetched into registers), writes the partial tile, and a second
// kernel sums the P partials in a fixed order.  Deterministic: the same
// shapes always use the same chunking and summation order.
#include "gala_internal.h"

namespace gala {
namespace {

constexpr int kRows = 32;    // rows staged in LDS per step
constexpr int kPad = 4;
constexpr int kRedLanes = 64; // lanes (one wave) per output in the partial-sum reduction

// One TK x TM (k, m) tile of one row chunk.  Lane layout: (TK/4) x (TM/4) = 256 lanes,
// each owning a 4x4 register block; the next 32-row step is loaded into registers while
// the current one is consumed from LDS.
template <int TK, int TM>
__global__ __launch_bounds__(kBlock) void k_tn_partial(int64_t N, int32_t K, int32_t M,
                                                       const float *__restrict__ X, int64_t ldx,
                                                       const float *__restrict__ dY, int64_t ldy,
                                                       int64_t rows_per_chunk,
                                                       float *__restrict__ part,
                                                       float *__restrict__ bpart) {
    static_assert((TK / 4) * (TM / 4) == kBlock, "one 4x4 block per lane");
    constexpr int LX = kRows * TK / kBlock, LY = kRows * TM / kBlock;  // staged values per lane
    __shared__ float sx[kRows][TK + kPad];
    __shared__ float sy[kRows][TM + kPad];
    const int t = threadIdx.x;
    const int tk = (t % (TK / 4)) * 4, tm = (t / (TK / 4)) * 4;
    const int k0 = blockIdx.x * TK, m0 = blockIdx.y * TM;
    const int64_t p = blockIdx.z;
    const int64_t r0 = p * rows_per_chunk;
    const int64_t r1 = r0 + rows_per_chunk < N ? r0 + rows_per_chunk : N;
    float acc[4][4] = {};
    float bacc[4] = {};
    float rx[LX], ry[LY];
    auto fetch = [&](int64_t rb) {
#pragma unroll
        for (int i = 0; i < LX; ++i) {
            const int e = t + i * kBlock, r = e / TK, c = e % TK;
            const int64_t row = rb + r;
            rx[i] = (row < r1 && k0 + c < K) ? X[row * ldx + k0 + c] : 0.0f;
        }
#pragma unroll
        for (int i = 0; i < LY; ++i) {
            const int e = t + i * kBlock, r = e / TM, c = e % TM;
            const int64_t row = rb + r;
            ry[i] = (row < r1 && m0 + c < M) ? dY[row * ldy + m0 + c] : 0.0f;
        }
    };
    if (r0 < r1) fetch(r0);
    for (int64_t rb = r0; rb < r1; rb += kRows) {
#pragma unroll
        for (int i = 0; i < LX; ++i) {
            const int e = t + i * kBlock;
            sx[e / TK][e % TK] = rx[i];
        }
#pragma unroll
        for (int i = 0; i < LY; ++i) {
            const int e = t + i * kBlock;
            sy[e / TM][e % TM] = ry[i];
        }
        __syncthreads();
        if (rb + kRows < r1) fetch(rb + kRows);  // in flight during the FMAs below
#pragma unroll 8
        for (int r = 0; r < kRows; ++r) {
            const float4 xv = *reinterpret_cast<const float4 *>(&sx[r][tk]);
            const float4 yv = *reinterpret_cast<const float4 *>(&sy[r][tm]);
            const float xs[4] = {xv.x, xv.y, xv.z, xv.w};
            const float ys[4] = {yv.x, yv.y, yv.z, yv.w};
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(ys[i], xs[j], acc[i][j]);
#pragma unroll
            for (int i = 0; i < 4; ++i) bacc[i] += ys[i];
        }
        __syncthreads();
    }
    // partial tile [M][K] of chunk p
    float *out = part + p * (int64_t)M * K;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + tm + i;
        if (m >= M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = k0 + tk + j;
            if (k < K) out[(int64_t)m * K + k] = acc[i][j];
        }
    }
    if (bpart && blockIdx.x == 0 && tk == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (m0 + tm + i < M) bpart[p * M + m0 + tm + i] = bacc[i];
    }
}

// out[i] (+)= sum_p part[p][i]: one wave per output; lane g sums the residue class
// p = g mod 64 in order (8 loads in flight), then a fixed xor butterfly adds the 64 lane
// sums (deterministic for given shapes).  One wave per output keeps the ~1000 partials
// of a chunk-split contraction from serialising in a handful of lanes.
__global__ __launch_bounds__(kBlock) void k_tn_reduce(int64_t count, int64_t P,
                                                      const float *__restrict__ part,
                                                      float *__restrict__ out, int accum) {
    constexpr int kOut = kBlock / kRedLanes;
    const int g = threadIdx.x % kRedLanes;
    const int64_t i = (int64_t)blockIdx.x * kOut + threadIdx.x / kRedLanes;
    if (i >= count) return;  // whole waves exit together
    float s = 0.0f;
    int64_t p = g;
    for (; p + 7 * kRedLanes < P; p += 8 * kRedLanes) {
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = part[(p + k * kRedLanes) * count + i];
#pragma unroll
        for (int k = 0; k < 8; ++k) s += v[k];
    }
    for (; p < P; p += kRedLanes) s += part[p * count + i];
#pragma unroll
    for (int o = kRedLanes / 2; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
    if (g == 0) out[i] = accum ? out[i] + s : s;
}

struct Plan {
    int tk, tm;  // tile shape
    int tiles_k, tiles_m;
    int64_t P, rows_per_chunk;
};

Plan plan_for(int64_t N, int32_t K, int32_t M) {
    Plan pl;
    // narrow outputs (M <= 32, e.g. hidden 32 or 16) take a 128 x 32 tile: no idle lanes
    pl.tm = M <= 32 ? 32 : 64;
    pl.tk = M <= 32 ? 128 : 64;
    pl.tiles_k = (K + pl.tk - 1) / pl.tk;
    pl.tiles_m = (M + pl.tm - 1) / pl.tm;
    const int64_t tiles = (int64_t)pl.tiles_k * pl.tiles_m;
    // ~4 workgroups per CU in total, each chunk a multiple of the LDS step
    int64_t P = (1024 + tiles - 1) / tiles;
    const int64_t max_p = (N + kRows - 1) / kRows;
    if (P > max_p) P = max_p;
    if (P < 1) P = 1;
    int64_t rpc = (N + P - 1) / P;
    rpc = (rpc + kRows - 1) / kRows * kRows;
    P = (N + rpc - 1) / rpc;
    pl.P = P < 1 ? 1 : P;
    pl.rows_per_chunk = rpc < kRows ? kRows : rpc;
    return pl;
}

}  // namespace
}  // namespace gala

using namespace gala;

extern "C" int64_t gala_dense_grad_workspace(int64_t n_rows, int32_t K, int32_t M) {
    if (n_rows < 0 || K < 0 || M < 0) return -1;
    if (n_rows == 0 || K == 0 || M == 0) return 0;
    const Plan pl = plan_for(n_rows, K, M);
    return (int64_t)sizeof(float) * pl.P * ((int64_t)M * K + M);
}

extern "C" int gala_dense_grad_f32(int64_t n_rows, int32_t K, int32_t M, const float *X,
                                   int64_t ldx, const float *dY, int64_t ldy, float *dW,
                                   float *db, int32_t accumulate, void *workspace,
                                   int64_t workspace_bytes, void *stream) {
    if (n_rows < 0 || K < 0 || M < 0 || ldx < K || ldy < M) return GALA_ERR_INVALID_ARG;
    if (K == 0 || M == 0) return GALA_OK;
    if (!dW) return GALA_ERR_INVALID_ARG;
    hipStream_t hs = (hipStream_t)stream;
    if (n_rows == 0) {
        // empty contraction: zero gradients (or leave accumulators untouched)
        if (!accumulate) {
            if (hipMemsetAsync(dW, 0, sizeof(float) * (size_t)M * K, hs) != hipSuccess ||
                (db && hipMemsetAsync(db, 0, sizeof(float) * (size_t)M, hs) != hipSuccess))
                return launch_status();
        }
        return GALA_OK;
    }
    if (!X || !dY || !workspace) return GALA_ERR_INVALID_ARG;
    const Plan pl = plan_for(n_rows, K, M);
    if (workspace_bytes < (int64_t)sizeof(float) * pl.P * ((int64_t)M * K + M))
        return GALA_ERR_INVALID_ARG;
    float *part = (float *)workspace;
    float *bpart = part + pl.P * (int64_t)M * K;
    const dim3 grid(pl.tiles_k, pl.tiles_m, (unsigned)pl.P);
    if (pl.tm == 32)
        hipLaunchKernelGGL((k_tn_partial<128, 32>), grid, dim3(kBlock), 0, hs, n_rows, K, M, X, ldx,
                           dY, ldy, pl.rows_per_chunk, part, db ? bpart : nullptr);
    else
        hipLaunchKernelGGL((k_tn_partial<64, 64>), grid, dim3(kBlock), 0, hs, n_rows, K, M, X, ldx,
                           dY, ldy, pl.rows_per_chunk, part, db ? bpart : nullptr);
    int st = launch_status();
    if (st) return st;
    const int64_t cw = (int64_t)M * K;
    constexpr int kOut = kBlock / kRedLanes;
    hipLaunchKernelGGL(k_tn_reduce, dim3((unsigned)((cw + kOut - 1) / kOut)), dim3(kBlock), 0,
                       hs, cw, pl.P, part, dW, accumulate);
    st = launch_status();
    if (st || !db) return st;
    hipLaunchKernelGGL(k_tn_reduce, dim3((unsigned)((M + kOut - 1) / kOut)), dim3(kBlock), 0,
                       hs, (int64_t)M, pl.P, bpart, db, accumulate);
    return launch_status();
}
