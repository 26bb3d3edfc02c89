// dense.hip — weight / bias gradients of the FFN (FFN_OP) for tall-skinny node matrices.
//
// The generated programs' FFNs are torch Linear layers on [N, K] node features with
// N = 10^5..10^8 and K, M <= a few hundred (gala.cu:415-420, common.h:1188-1242).  Their
// backward needs dW[m, k] = sum_n dY[n, m] X[n, k] and db[m] = sum_n dY[n, m]: a GEMM whose
// contraction runs over the N rows.  Measured on the Products GCN program before this
// kernel, torch's bias reduction over dim 0 took 18.6 ms and the weight GEMM 3.3 ms, for
// 1.3 GB of input that HBM streams in ~0.2 ms (tools/dense_bench.py times both).  Here the rows are split into P chunks
// (split-K) and a second kernel sums the P partials in a fixed order:
//  * k_tn_mfma: every wave owns a (32 WM) x (32 WK) tile of dW for one row chunk and runs
//    it on the exact-f32 matrix cores (v_mfma_f32_32x32x2_f32: each instruction takes two
//    rows, operands straight from global memory -- lane l reads dY[n][m0 + l%32] and
//    X[n][k0 + l%32] of row n = 2s + l/32, both 128-B coalesced -- no LDS); consecutive
//    waves share a chunk, so a row's bytes are fetched once and re-read from cache;
//  * k_tn_lds: M and K > 64 with float4 rows, 128 (or 192) x 128 block tiles whose row stages come
//    through LDS, double-buffered (see below);
//  * k_tn_skinny: M <= 4 (the attention Linears, out = 1), lanes over K, see below.
// Deterministic: the same shapes always use the same chunking and summation order (an
// f32 MFMA is bit-for-bit a row-ordered fmaf chain).
#include "gala_internal.h"

namespace gala {
namespace {

constexpr int kStep = 2;      // rows per MFMA (the K of 32x32x2)
// MFMA steps whose operand loads are issued together: 4 for the small (pipelined) wave
// tiles, 8 for 2 x 2 tiles, which wait for one batch at a time and need the longer run of
// MFMAs per wait to keep the matrix cores busy at ~3 waves per SIMD
template <int WM, int WK>
constexpr int in_flight() { return WM * WK < 4 ? 4 : 8; }
constexpr int kRowAlign = 16;  // rows per chunk: a multiple of every kStep * in_flight

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int WM, int WK>
__global__ __launch_bounds__(kBlock) void k_tn_mfma(int64_t N, int32_t K, int32_t M,
                                                    const float *__restrict__ X, int64_t ldx,
                                                    const float *__restrict__ dY, int64_t ldy,
                                                    int64_t rows_per_chunk, int32_t tiles_k,
                                                    int32_t n_tg, int64_t n_work,
                                                    float *__restrict__ part,
                                                    float *__restrict__ bpart) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t w = (int64_t)blockIdx.x * (kBlock / kWave) + threadIdx.x / kWave;
    if (w >= n_work) return;  // whole waves; no block-level synchronisation
    const int64_t chunk = w / n_tg;
    const int tg = (int)(w % n_tg);
    const int m0 = (tg / tiles_k) * 32 * WM, k0 = (tg % tiles_k) * 32 * WK;
    const int64_t r0 = chunk * rows_per_chunk;
    const int64_t r1 = r0 + rows_per_chunk < N ? r0 + rows_per_chunk : N;
    const int li = lane & 31, lh = lane >> 5;
    constexpr int kInFlight = in_flight<WM, WK>();
    bool mv[WM], kv[WK];
    int64_t mo[WM], ko[WK];
#pragma unroll
    for (int a = 0; a < WM; ++a) {
        const int m = m0 + a * 32 + li;
        mv[a] = m < M;
        mo[a] = mv[a] ? m : 0;
    }
#pragma unroll
    for (int b = 0; b < WK; ++b) {
        const int k = k0 + b * 32 + li;
        kv[b] = k < K;
        ko[b] = kv[b] ? k : 0;
    }
    f32x16 acc[WM][WK];
#pragma unroll
    for (int a = 0; a < WM; ++a)
#pragma unroll
        for (int b = 0; b < WK; ++b) acc[a][b] = f32x16(0.0f);
    float bacc[WM] = {};
    // software-pipelined: the next kInFlight steps' operands are loaded while the current
    // ones feed the matrix cores
    float av[kInFlight][WM], bv[kInFlight][WK];
    auto load = [&](int64_t rb) {
#pragma unroll
        for (int u = 0; u < kInFlight; ++u) {
            const int64_t n = rb + kStep * u + lh;
            const bool ok = n < r1;
#pragma unroll
            for (int a = 0; a < WM; ++a) av[u][a] = (ok && mv[a]) ? dY[n * ldy + mo[a]] : 0.0f;
#pragma unroll
            for (int b = 0; b < WK; ++b) bv[u][b] = (ok && kv[b]) ? X[n * ldx + ko[b]] : 0.0f;
        }
    };
    // (2 x 2 wave tiles are matrix-core bound and keep their occupancy instead)
    constexpr bool kPipe = WM * WK < 4;
    if (kPipe && r0 < r1) load(r0);
    for (int64_t rb = r0; rb < r1; rb += kStep * kInFlight) {
        if (!kPipe) load(rb);
        float ca[kInFlight][WM], cb[kInFlight][WK];
#pragma unroll
        for (int u = 0; u < kInFlight; ++u) {
#pragma unroll
            for (int a = 0; a < WM; ++a) ca[u][a] = av[u][a];
#pragma unroll
            for (int b = 0; b < WK; ++b) cb[u][b] = bv[u][b];
        }
        if (kPipe && rb + kStep * kInFlight < r1) load(rb + kStep * kInFlight);
#pragma unroll
        for (int u = 0; u < kInFlight; ++u) {
#pragma unroll
            for (int a = 0; a < WM; ++a) {
                bacc[a] += ca[u][a];
#pragma unroll
                for (int b = 0; b < WK; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(ca[u][a], cb[u][b], acc[a][b], 0, 0, 0);
            }
        }
    }
    // C/D layout: column (k) = lane % 32, row (m) = (r & 3) + 8 (r >> 2) + 4 (lane / 32)
    float *out = part + chunk * (int64_t)M * K;
#pragma unroll
    for (int a = 0; a < WM; ++a)
#pragma unroll
        for (int b = 0; b < WK; ++b) {
            const int k = k0 + b * 32 + li;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                if (m < M && k < K) out[(int64_t)m * K + k] = acc[a][b][r];
            }
        }
    if (bpart && k0 == 0) {  // db: the two row parities (lane halves) of the k0 = 0 tile
#pragma unroll
        for (int a = 0; a < WM; ++a) {
            const float s2 = bacc[a] + __shfl_xor(bacc[a], 32, kWave);
            if (lh == 0 && mv[a]) bpart[chunk * M + mo[a]] = s2;
        }
    }
}

// Wide tiles (M > 64 and K > 64, every row a whole number of float4: config 5's 128 x 128
// and 128 x 172 layers): a block owns a BM (m) x 128 (k) tile of dW for one row chunk, and
// its 32-row (16 at BM = 192) stages of dY and X come through LDS -- one float4 load per lane and row piece,
// double-buffered, the next stage's loads in flight while the matrix cores work on this one.
// k_tn_mfma fed every MFMA operand by its own 4-B global load and waited out each batch
// (5.0 ms for 11 M x 128 x 128, 0.46 of the f32 matrix peak).  Wave w of the block owns the
// (BM / 2) x 64 quarter (m: w / 2, k: w % 2) as WT x 2 32x32x2 tiles; BM = 64 WT is 128, or
// 192 when that pads M less (M = 172: one 192 tile instead of two of 128, the second 44
// rows live).  A staged row of E floats sits at a stride of E + 32, so the two row halves of
// an operand read (lanes 0-31 row n, 32-63 row n + 1) fall in different banks.  Same partial
// layout and reduction as the other kernels.
constexpr int kLdsK = 128;    // k extent of a block tile
template <int WT>
struct LdsTile {
    static constexpr int R = WT == 2 ? 32 : 16;                // rows per stage
    static constexpr int BM = 64 * WT;                         // m extent of a block tile
    static constexpr int SY = BM + 32, SX = kLdsK + 32;        // staged row strides
    static constexpr int stage = R * (SY + SX);                // dY then X, floats
    static constexpr size_t bytes = 2 * stage * sizeof(float);  // double-buffered: 80 / 48 KB
    static constexpr int NY = R * BM / 4 / kBlock;             // float4 loads per thread and stage
    static constexpr int NX = R * kLdsK / 4 / kBlock;
};

template <int WT>
__global__ __launch_bounds__(kBlock) void k_tn_lds(int64_t N, int32_t K, int32_t M,
                                                   const float *__restrict__ X, int64_t ldx,
                                                   const float *__restrict__ dY, int64_t ldy,
                                                   int64_t rows_per_chunk, int32_t tiles_m, int32_t tiles_k,
                                                   float *__restrict__ part, float *__restrict__ bpart) {
    typedef LdsTile<WT> T;
    extern __shared__ float lds[];
    const int64_t chunk = blockIdx.x / (tiles_m * tiles_k);
    const int tg = (int)(blockIdx.x % (tiles_m * tiles_k));
    const int mB = (tg / tiles_k) * T::BM, kB = (tg % tiles_k) * kLdsK;
    const int64_t r0 = chunk * rows_per_chunk;
    const int64_t r1 = r0 + rows_per_chunk < N ? r0 + rows_per_chunk : N;
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
    const int li = lane & 31, lh = lane >> 5;
    const int mw = (wv >> 1) * 32 * WT, kw = (wv & 1) * 64;  // this wave's quarter of the tile
    // stage loads: float4 q = threadIdx.x + kBlock i of the stage's row-major image
    float4 ry[T::NY], rx[T::NX];
    auto gload = [&](int64_t rb) {
#pragma unroll
        for (int i = 0; i < T::NY; ++i) {
            const int q = threadIdx.x + kBlock * i, r = q / (T::BM / 4), c = (q % (T::BM / 4)) * 4;
            const int64_t n = rb + r;
            ry[i] = (n < r1 && mB + c < M) ? *reinterpret_cast<const float4 *>(dY + n * ldy + mB + c)
                                          : make_float4(0, 0, 0, 0);  // M a multiple of 4: whole vectors
        }
#pragma unroll
        for (int i = 0; i < T::NX; ++i) {
            const int q = threadIdx.x + kBlock * i, r = q / (kLdsK / 4), c = (q % (kLdsK / 4)) * 4;
            const int64_t n = rb + r;
            rx[i] = (n < r1 && kB + c < K) ? *reinterpret_cast<const float4 *>(X + n * ldx + kB + c)
                                          : make_float4(0, 0, 0, 0);
        }
    };
    auto swrite = [&](float *st) {
#pragma unroll
        for (int i = 0; i < T::NY; ++i) {
            const int q = threadIdx.x + kBlock * i, r = q / (T::BM / 4), c = (q % (T::BM / 4)) * 4;
            *reinterpret_cast<float4 *>(st + r * T::SY + c) = ry[i];
        }
#pragma unroll
        for (int i = 0; i < T::NX; ++i) {
            const int q = threadIdx.x + kBlock * i, r = q / (kLdsK / 4), c = (q % (kLdsK / 4)) * 4;
            *reinterpret_cast<float4 *>(st + T::R * T::SY + r * T::SX + c) = rx[i];
        }
    };
    f32x16 acc[WT][2];
#pragma unroll
    for (int a = 0; a < WT; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = f32x16(0.0f);
    float bacc[WT] = {};
    const bool live = mB + mw < M && kB + kw < K;  // wave-uniform
    if (r0 < r1) gload(r0);
    int buf = 0;
    for (int64_t rb = r0; rb < r1; rb += T::R) {
        float *st = lds + buf * T::stage;
        swrite(st);
        __syncthreads();
        if (rb + T::R < r1) gload(rb + T::R);
        buf ^= 1;
        if (!live) continue;  // a quarter wholly past M or K
        const float *ys = st + lh * T::SY + mw + li;
        const float *xs = st + T::R * T::SY + lh * T::SX + kw + li;
#pragma unroll 4
        for (int s2 = 0; s2 < T::R; s2 += 2) {
            float av[WT], bv[2];
#pragma unroll
            for (int a = 0; a < WT; ++a) av[a] = ys[s2 * T::SY + a * 32];
#pragma unroll
            for (int b = 0; b < 2; ++b) bv[b] = xs[s2 * T::SX + b * 32];
#pragma unroll
            for (int a = 0; a < WT; ++a) {
                bacc[a] += av[a];
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[a], bv[b], acc[a][b], 0, 0, 0);
            }
        }
    }
    // C/D layout: column (k) = lane % 32, row (m) = (r & 3) + 8 (r >> 2) + 4 (lane / 32)
    float *out = part + chunk * (int64_t)M * K;
#pragma unroll
    for (int a = 0; a < WT; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const int k = kB + kw + b * 32 + li;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = mB + mw + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                if (m < M && k < K) out[(int64_t)m * K + k] = acc[a][b][r];
            }
        }
    if (bpart && kB == 0 && kw == 0) {  // db: the two row parities (lane halves)
#pragma unroll
        for (int a = 0; a < WT; ++a) {
            const float s2 = bacc[a] + __shfl_xor(bacc[a], 32, kWave);
            const int m = mB + mw + a * 32 + li;
            if (lh == 0 && m < M) bpart[chunk * M + m] = s2;
        }
    }
}

// ---- FFN forward: Y[N, M] = X[N, K] W^T + b on the matrix cores ----------------------
// A block walks groups of 4 row tiles (32 rows each, one per wave) grid-stride.  W^T lives
// in LDS for the whole block (K*M <= kFwdMaxKM floats); each wave stages its 32 x K tile of
// X in LDS with coalesced (float4 where aligned) loads -- consecutive rows are contiguous --
// at an odd row stride, so the MFMA operand reads (lane l: row l%32, k = 2s + l/32) are
// bank-conflict free.  One wave owns all M columns (WM tiles of 32); accumulators start at
// the bias, and each 32x32 C tile is stored with 32 lanes on 32 consecutive columns of a row.
constexpr int kFwdMaxKM = 24576;  // W^T floats in LDS (96 KB; past 64 KB the launch opts in)
constexpr size_t kFwdMaxLds = 160 * 1024;  // gfx950's LDS per CU

template <int WM, int V>
__global__ __launch_bounds__(kBlock) void k_ffn_fwd(int64_t N, int32_t K, int32_t M,
                                                    const float *__restrict__ X, int64_t ldx,
                                                    const float *__restrict__ W,
                                                    const float *__restrict__ bias,
                                                    float *__restrict__ Y, int64_t ldy) {
    extern __shared__ float smem[];
    constexpr int Mp = 32 * WM;
    const int Kp = (K + 1) & ~1;       // whole MFMA steps (an odd tail k reads zeros)
    const int KS = Kp + 1;             // odd LDS row stride of the X tiles
    float *wt = smem;                  // wt[k * Mp + m] = W[m][k], zero padded
    for (int t = threadIdx.x; t < Kp * Mp; t += kBlock) {
        const int k = t / Mp, m = t % Mp;
        wt[t] = (k < K && m < M) ? W[(int64_t)m * K + k] : 0.0f;
    }
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
    const int li = lane & 31, lh = lane >> 5;
    float *xs = smem + Kp * Mp + wv * 32 * KS;
    for (int t = lane; t < 32 * KS; t += kWave) xs[t] = 0.0f;  // the padding column stays 0
    __syncthreads();
    float bv[WM];
#pragma unroll
    for (int a = 0; a < WM; ++a) {
        const int m = a * 32 + li;
        bv[a] = (bias && m < M) ? bias[m] : 0.0f;
    }
    const int64_t tiles = (N + 31) / 32;
    const int Kq = (K + V - 1) / V;    // V-float vectors per row
    for (int64_t g0 = (int64_t)blockIdx.x * 4; g0 < tiles; g0 += (int64_t)gridDim.x * 4) {
        const int64_t n0 = (g0 + wv) * 32;
        // stage this wave's 32 x K tile (rows past N read as zeros)
        for (int t = lane; t < 32 * Kq; t += kWave) {
            const int r = t / Kq, c = (t - r * Kq) * V;
            const int64_t n = n0 + r;
            float v[V];
            if (V == 4 && n < N) {
                const float4 q = *reinterpret_cast<const float4 *>(X + n * ldx + c);
                v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
            } else {
#pragma unroll
                for (int i = 0; i < V; ++i) v[i] = (n < N && c + i < K) ? X[n * ldx + c + i] : 0.0f;
            }
#pragma unroll
            for (int i = 0; i < V; ++i) xs[r * KS + c + i] = v[i];
        }
        __syncthreads();
        f32x16 acc[WM];
#pragma unroll
        for (int a = 0; a < WM; ++a) acc[a] = f32x16(bv[a]);
        const float *xrow = xs + li * KS + lh;
        const float *wcol = wt + lh * Mp + li;
        for (int s2 = 0; s2 < Kp; s2 += 2) {
            const float xa = xrow[s2];
#pragma unroll
            for (int a = 0; a < WM; ++a)
                acc[a] = __builtin_amdgcn_mfma_f32_32x32x2f32(xa, wcol[s2 * Mp + a * 32], acc[a], 0, 0, 0);
        }
        // C/D: column (m) = lane % 32, row (n) = (r & 3) + 8 (r >> 2) + 4 (lane / 32)
#pragma unroll
        for (int a = 0; a < WM; ++a) {
            const int m = a * 32 + li;
            if (m >= M) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t nr = n0 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                if (nr < N) Y[nr * ldy + m] = acc[a][r];
            }
        }
        __syncthreads();  // the tile buffers are refilled next round
    }
}

// Narrow outputs (M <= 4: the attention Linears, out = 1): a (k, m) tile would leave most
// lanes idle and the kernel latency-bound.  Here KL lanes span a row's K columns (CH per
// lane past 64), a wave covers 64/KL rows per step with 4 steps' loads in flight, and every
// lane keeps M x CH accumulators; the block's lanes and waves are then summed through LDS
// in a fixed order into the chunk's partial [M][K] (+ [M] bias) -- same partial layout and
// reduction kernel as the tiles.
template <int MM, int KL, int CH>
__global__ __launch_bounds__(kBlock) void k_tn_skinny(int64_t N, int32_t K, int32_t M,
                                                      const float *__restrict__ X, int64_t ldx,
                                                      const float *__restrict__ dY, int64_t ldy,
                                                      int64_t rows_per_chunk,
                                                      float *__restrict__ part,
                                                      float *__restrict__ bpart) {
    constexpr int RPW = kWave / KL;              // rows per wave step
    constexpr int RPB = RPW * (kBlock / kWave);  // rows per block step
    constexpr int U = 4;                         // block steps in flight
    __shared__ float red[RPB][MM][KL * CH + 1];
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
    const int kl = lane % KL, rs = wv * RPW + lane / KL;
    const int64_t p = blockIdx.x;
    const int64_t r0 = p * rows_per_chunk;
    const int64_t r1 = r0 + rows_per_chunk < N ? r0 + rows_per_chunk : N;
    float acc[MM][CH] = {};
    float bacc[MM] = {};
    for (int64_t rb = r0 + rs; rb < r1; rb += (int64_t)U * RPB) {
        float x[U][CH], y[U][MM];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t row = rb + (int64_t)u * RPB;
            const bool ok = row < r1;
#pragma unroll
            for (int j = 0; j < CH; ++j) {
                const int k = j * KL + kl;
                x[u][j] = (ok && k < K) ? X[row * ldx + k] : 0.0f;
            }
#pragma unroll
            for (int m = 0; m < MM; ++m) y[u][m] = (ok && m < M) ? dY[row * ldy + m] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int m = 0; m < MM; ++m) {
#pragma unroll
                for (int j = 0; j < CH; ++j) acc[m][j] = fmaf(y[u][m], x[u][j], acc[m][j]);
                bacc[m] += y[u][m];
            }
    }
#pragma unroll
    for (int m = 0; m < MM; ++m)
#pragma unroll
        for (int j = 0; j < CH; ++j) red[rs][m][j * KL + kl] = acc[m][j];
    __syncthreads();
    // thread t sums output (m, k) = t over the RPB row slots in order
    for (int o = threadIdx.x; o < M * K; o += kBlock) {
        const int m = o / K, k = o % K;
        float s = 0.0f;
        for (int r = 0; r < RPB; ++r) s += red[r][m][k];
        part[p * (int64_t)M * K + o] = s;
    }
    if (bpart) {
        __syncthreads();
        if (kl == 0)
#pragma unroll
            for (int m = 0; m < MM; ++m) red[rs][m][0] = bacc[m];
        __syncthreads();
        if (threadIdx.x < M) {
            float s = 0.0f;
            for (int r = 0; r < RPB; ++r) s += red[r][threadIdx.x][0];
            bpart[p * M + threadIdx.x] = s;
        }
    }
}

// out[i] (+)= sum_p part[p][i] in two coalesced passes (threads along i, so a block reads
// 1 KB of one partial row per load): pass A sums runs of kRedChain partials into
// part2[q][i], pass B sums the runs in order (pass A is skipped when P <= kRedChain).
// Deterministic for given shapes.
constexpr int kRedChain = 64;

__device__ __forceinline__ float sum_strided(const float *__restrict__ a, int64_t stride,
                                             int64_t n) {
    float s = 0.0f;
    int64_t j = 0;
    for (; j + 8 <= n; j += 8) {
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = a[(j + k) * stride];
#pragma unroll
        for (int k = 0; k < 8; ++k) s += v[k];
    }
    for (; j < n; ++j) s += a[j * stride];
    return s;
}

__global__ __launch_bounds__(kBlock) void k_tn_reduce_a(int64_t count, int64_t P,
                                                        const float *__restrict__ part,
                                                        float *__restrict__ part2) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= count) return;
    const int64_t p0 = (int64_t)blockIdx.y * kRedChain;
    const int64_t n = P - p0 < kRedChain ? P - p0 : kRedChain;
    part2[(int64_t)blockIdx.y * count + i] = sum_strided(part + p0 * count + i, count, n);
}

__global__ __launch_bounds__(kBlock) void k_tn_reduce_b(int64_t count, int64_t Q,
                                                        const float *__restrict__ part2,
                                                        float *__restrict__ out, int accum) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= count) return;
    const float s = sum_strided(part2 + i, count, Q);
    out[i] = accum ? out[i] + s : s;
}

struct Plan {
    bool skinny;      // M <= 4 and K <= 256: k_tn_skinny; else k_tn_mfma
    bool staged;      // M, K > 64, float4 rows: k_tn_lds (tiles_k / n_tg: its BM x 128 tiles)
    int wt;           // k_tn_lds: BM = 64 wt (2 or 3)
    int wm, wk;       // MFMA wave tile: (32 wm) x (32 wk)
    int tiles_k, n_tg;  // wave tiles along K, per chunk
    int64_t P, rows_per_chunk;
};

constexpr int kSkinnyM = 4, kSkinnyK = 256;

Plan plan_for(int64_t N, int32_t K, int32_t M, bool vec4) {
    Plan pl{};
    pl.skinny = M <= kSkinnyM && K <= kSkinnyK;
    pl.staged = !pl.skinny && vec4 && M > 64 && K > 64;
    int64_t target;  // chunks
    int64_t align;   // rows per chunk: a multiple of the kernel's row step
    if (pl.staged) {  // the m extent that pads M least; ~2 blocks per CU
        const int64_t m128 = (M + 127) / 128 * 128, m192 = (M + 191) / 192 * 192;
        pl.wt = m192 < m128 ? 3 : 2;
        const int bm = 64 * pl.wt;
        pl.tiles_k = (K + kLdsK - 1) / kLdsK;
        pl.n_tg = pl.tiles_k * ((M + bm - 1) / bm);
        target = (512 + pl.n_tg - 1) / pl.n_tg;
        align = 32;  // whole stages of either tile
    } else if (pl.skinny) {  // ~4 blocks per CU, chunks of whole block steps (4 x 4 waves x rows)
        pl.tiles_k = pl.n_tg = 1;
        target = 1024;
        align = 64;
    } else {          // ~8192 waves (32 per CU), consecutive waves on one chunk
        pl.wm = M > 32 ? 2 : 1;
        pl.wk = K > 32 ? 2 : 1;
        pl.tiles_k = (K + 32 * pl.wk - 1) / (32 * pl.wk);
        pl.n_tg = pl.tiles_k * ((M + 32 * pl.wm - 1) / (32 * pl.wm));
        target = (8192 + pl.n_tg - 1) / pl.n_tg;
        align = kRowAlign;
    }
    int64_t rpc = (N + target - 1) / target;
    rpc = (rpc + align - 1) / align * align;
    pl.rows_per_chunk = rpc < align ? align : rpc;
    pl.P = (N + pl.rows_per_chunk - 1) / pl.rows_per_chunk;
    if (pl.P < 1) pl.P = 1;
    return pl;
}

// runs of kRedChain partials summed by pass A (1: pass B alone)
int64_t red_runs(int64_t P) { return P <= kRedChain ? 1 : (P + kRedChain - 1) / kRedChain; }

int reduce_partials(int64_t count, int64_t P, const float *part, float *part2, float *out,
                    int accum, hipStream_t hs) {
    const unsigned gx = (unsigned)((count + kBlock - 1) / kBlock);
    const float *src = part;
    int64_t n = P;
    if (P > kRedChain) {
        hipLaunchKernelGGL(k_tn_reduce_a, dim3(gx, (unsigned)red_runs(P)), dim3(kBlock), 0, hs,
                           count, P, part, part2);
        src = part2;
        n = red_runs(P);
    }
    hipLaunchKernelGGL(k_tn_reduce_b, dim3(gx), dim3(kBlock), 0, hs, count, n, src, out, accum);
    return launch_status();
}

}  // namespace
}  // namespace gala

using namespace gala;

extern "C" int64_t gala_dense_grad_workspace(int64_t n_rows, int32_t K, int32_t M) {
    if (n_rows < 0 || K < 0 || M < 0) return -1;
    if (n_rows == 0 || K == 0 || M == 0) return 0;
    // the workspace bound of either plan (the float4 test needs the operands)
    const Plan a = plan_for(n_rows, K, M, false), b = plan_for(n_rows, K, M, true);
    const int64_t P = a.P + red_runs(a.P) > b.P + red_runs(b.P) ? a.P + red_runs(a.P) : b.P + red_runs(b.P);
    return (int64_t)sizeof(float) * P * ((int64_t)M * K + M);
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
    const bool vec4 = K % 4 == 0 && M % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && ((uintptr_t)X % 16) == 0 &&
                      ((uintptr_t)dY % 16) == 0;
    const Plan pl = plan_for(n_rows, K, M, vec4);
    const int64_t Q = red_runs(pl.P);
    if (workspace_bytes < (int64_t)sizeof(float) * (pl.P + Q) * ((int64_t)M * K + M))
        return GALA_ERR_INVALID_ARG;
    float *part = (float *)workspace;
    float *bpart = part + pl.P * (int64_t)M * K;
    float *part2 = bpart + pl.P * (int64_t)M;
    float *bpart2 = part2 + Q * (int64_t)M * K;
    if (pl.skinny) {
        // KL lanes per row: the smallest power of two covering K, at most 64 (CH past it)
        int kl = 1;
        while (kl < K && kl < 64) kl <<= 1;
        const int ch = (K + 63) / 64;
        const dim3 g1((unsigned)pl.P);
        float *bp = db ? bpart : nullptr;
#define GALA_SK(KL, CH) hipLaunchKernelGGL((k_tn_skinny<kSkinnyM, KL, CH>), g1, dim3(kBlock), 0, hs, n_rows, \
                                           K, M, X, ldx, dY, ldy, pl.rows_per_chunk, part, bp)
        if (kl <= 8) GALA_SK(8, 1);
        else if (kl == 16) GALA_SK(16, 1);
        else if (kl == 32) GALA_SK(32, 1);
        else if (ch == 1) GALA_SK(64, 1);
        else if (ch == 2) GALA_SK(64, 2);
        else if (ch == 3) GALA_SK(64, 3);
        else GALA_SK(64, 4);
#undef GALA_SK
    } else if (pl.staged) {
#define GALA_LDS(WT)                                                                                        \
    do {                                                                                                    \
        static const hipError_t opted = hipFuncSetAttribute((const void *)k_tn_lds<WT>,                     \
                                                            hipFuncAttributeMaxDynamicSharedMemorySize,     \
                                                            (int)LdsTile<WT>::bytes);                       \
        (void)opted;                                                                                        \
        hipLaunchKernelGGL(k_tn_lds<WT>, dim3((unsigned)(pl.P * pl.n_tg)), dim3(kBlock), LdsTile<WT>::bytes, hs, \
                           n_rows, K, M, X, ldx, dY, ldy, pl.rows_per_chunk, pl.n_tg / pl.tiles_k, pl.tiles_k, \
                           part, db ? bpart : nullptr);                                                     \
    } while (0)
        if (pl.wt == 3) GALA_LDS(3);
        else GALA_LDS(2);
#undef GALA_LDS
    } else {
        const int64_t n_work = pl.P * pl.n_tg;
        const dim3 g((unsigned)((n_work + kBlock / kWave - 1) / (kBlock / kWave)));
        float *bp = db ? bpart : nullptr;
#define GALA_MF(WM, WK) hipLaunchKernelGGL((k_tn_mfma<WM, WK>), g, dim3(kBlock), 0, hs, n_rows, K, M, X, ldx, \
                                           dY, ldy, pl.rows_per_chunk, pl.tiles_k, pl.n_tg, n_work, part, bp)
        if (pl.wm == 1 && pl.wk == 1) GALA_MF(1, 1);
        else if (pl.wm == 1) GALA_MF(1, 2);
        else if (pl.wk == 1) GALA_MF(2, 1);
        else GALA_MF(2, 2);
#undef GALA_MF
    }
    int st = launch_status();
    if (st) return st;
    st = reduce_partials((int64_t)M * K, pl.P, part, part2, dW, accumulate, hs);
    if (st || !db) return st;
    return reduce_partials((int64_t)M, pl.P, bpart, bpart2, db, accumulate, hs);
}

extern "C" int gala_ffn_fwd_f32(int64_t n_rows, int32_t K, int32_t M, const float *X, int64_t ldx,
                                const float *W, const float *b, float *Y, int64_t ldy,
                                void *stream) {
    if (n_rows < 0 || K < 0 || M < 0 || ldx < K || ldy < M) return GALA_ERR_INVALID_ARG;
    if (n_rows == 0 || M == 0) return GALA_OK;
    const int wm = (M + 31) / 32;
    if (wm > 8 || (int64_t)((K + 1) & ~1) * 32 * wm > kFwdMaxKM) return GALA_ERR_UNSUPPORTED;
    if (!Y || (K > 0 && (!X || !W))) return GALA_ERR_INVALID_ARG;
    const int64_t tiles = (n_rows + 31) / 32;
    int64_t blocks = (tiles + 3) / 4;
    if (blocks > 256 * 4) blocks = 256 * 4;  // blocks then walk 4-tile groups grid-stride
    const int Kp = (K + 1) & ~1;
    const size_t lds = sizeof(float) * ((size_t)Kp * 32 * wm + 4 * 32 * (size_t)(Kp + 1));
    if (lds > kFwdMaxLds) return GALA_ERR_UNSUPPORTED;
    const bool v4 = K % 4 == 0 && ldx % 4 == 0 && ((uintptr_t)X % 16) == 0;
    hipStream_t hs = (hipStream_t)stream;
#define GALA_FF(WMV)                                                                                          \
    do {                                                                                                  \
        static const hipError_t o4 = hipFuncSetAttribute((const void *)k_ffn_fwd<WMV, 4>,                 \
                                                         hipFuncAttributeMaxDynamicSharedMemorySize,      \
                                                         (int)kFwdMaxLds);                                \
        static const hipError_t o1 = hipFuncSetAttribute((const void *)k_ffn_fwd<WMV, 1>,                 \
                                                         hipFuncAttributeMaxDynamicSharedMemorySize,      \
                                                         (int)kFwdMaxLds);                                \
        (void)o4;                                                                                         \
        (void)o1;                                                                                         \
        if (v4)                                                                                           \
            hipLaunchKernelGGL((k_ffn_fwd<WMV, 4>), dim3((unsigned)blocks), dim3(kBlock), lds, hs, n_rows, K, M, \
                               X, ldx, W, b, Y, ldy);                                                     \
        else                                                                                              \
            hipLaunchKernelGGL((k_ffn_fwd<WMV, 1>), dim3((unsigned)blocks), dim3(kBlock), lds, hs, n_rows, K, M, \
                               X, ldx, W, b, Y, ldy);                                                     \
    } while (0)
    switch (wm) {
        case 1: GALA_FF(1); break;
        case 2: GALA_FF(2); break;
        case 3: GALA_FF(3); break;
        case 4: GALA_FF(4); break;
        case 5: GALA_FF(5); break;
        case 6: GALA_FF(6); break;
        case 7: GALA_FF(7); break;
        default: GALA_FF(8); break;
    }
#undef GALA_FF
    return launch_status();
}
