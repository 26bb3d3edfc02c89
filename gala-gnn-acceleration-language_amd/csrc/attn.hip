// attn.hip -- the per-head attention logits of the multi-head GAT layer and their input
// gradient, for gfx950.
//
// With galac's gat_heads(H) the DSL's attnL = dsl.nn.ffn(res, out=1) is one Linear(D, 1)
// per head (tests/GALA-DSL/gat/Products/h100.txt:8-9 is its one-head form; the reference
// runs it as a torch::nn::Linear, common.h:1188-1242):
//     out[r, h] = <X[r, hD:(h+1)D], w[hD:(h+1)D]> + b[h]
// and its backward puts g[r, h] * w[hD:(h+1)D] into dX's head slice.  As torch ops these
// are a broadcast product into an [N, H, D] temporary plus a reduction (forward) and two
// more [N, F] passes (backward); here each is one pass over the rows.
//
// Forward layout: HW = D / VEC lanes per (row, head) pair (a power of two up to 64), each
// lane one VEC-wide slice, so a wave reads 64 consecutive vectors (contiguous rows);
// the pair's dot is each lane's fma chain over its slice, then an xor butterfly over the
// HW lanes (deterministic); a head width that is no power of two of vectors (D = 47) takes
// the next power of two of lanes, the ones past D idle.  Wider heads: one thread per pair, a
// sequential chain.
// Backward: one thread per VEC-wide vector of dX, consecutive threads on consecutive
// vectors (full-line stores).
#include "gala_internal.h"

namespace gala {

template <int VEC>
struct AVec;
template <>
struct AVec<1> { typedef float T; };
template <>
struct AVec<2> { typedef float T __attribute__((ext_vector_type(2))); };
template <>
struct AVec<4> { typedef float T __attribute__((ext_vector_type(4))); };

template <int VEC, int HW>
__global__ __launch_bounds__(kBlock) void k_head_attn_group(int64_t n_rows, int32_t H, int32_t D, const float *X,
                                                            int64_t ldx, const float *w, const float *b, float *out) {
    typedef typename AVec<VEC>::T V;
    const int64_t pair = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / HW;
    const int gl = threadIdx.x & (HW - 1);
    if (pair >= n_rows * H) return;  // whole groups leave together
    const int64_t r = pair / H;
    const int h = (int)(pair - r * H);
    // lanes past the head's D / VEC vectors (HW rounded up to a power of two) add nothing
    const bool live = gl * VEC < D;
    const int64_t c = (int64_t)h * D + (live ? gl * VEC : 0);
    const V x = *reinterpret_cast<const V *>(X + r * ldx + c);
    const V v = *reinterpret_cast<const V *>(w + c);
    float acc = 0.0f;
#pragma unroll
    for (int i = 0; i < VEC; ++i)
        acc = fmaf(reinterpret_cast<const float *>(&x)[i], reinterpret_cast<const float *>(&v)[i], acc);
    acc = group_sum<HW>(live ? acc : 0.0f);
    if (gl == 0) out[pair] = b ? __fadd_rn(acc, b[h]) : acc;
}

template <int VEC>
__global__ __launch_bounds__(kBlock) void k_head_attn(int64_t n_rows, int32_t H, int32_t D, const float *X,
                                                      int64_t ldx, const float *w, const float *b, float *out) {
    typedef typename AVec<VEC>::T V;
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= n_rows * H) return;
    const int64_t r = t / H;
    const int h = (int)(t - r * H);
    const float *xr = X + r * ldx + (int64_t)h * D;
    const float *wh = w + (int64_t)h * D;
    float acc = 0.0f;
    for (int d = 0; d < D; d += VEC) {
        const V x = *reinterpret_cast<const V *>(xr + d);
        const V v = *reinterpret_cast<const V *>(wh + d);
#pragma unroll
        for (int i = 0; i < VEC; ++i)
            acc = fmaf(reinterpret_cast<const float *>(&x)[i], reinterpret_cast<const float *>(&v)[i], acc);
    }
    out[t] = b ? __fadd_rn(acc, b[h]) : acc;
}

// dX[r, c] (+)= g[r, c / D] * w[c], one thread per vector
template <int VEC>
__global__ __launch_bounds__(kBlock) void k_head_attn_bwd(int64_t n_rows, int32_t F, int32_t H, int32_t D,
                                                          const float *g, const float *w, float *dX,
                                                          int64_t lddx, int32_t accumulate) {
    typedef typename AVec<VEC>::T V;
    const int32_t L = F / VEC;
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= n_rows * L) return;
    const int64_t r = t / L;
    const int32_t c = (int32_t)(t - r * L) * VEC;
    const float gv = g[r * H + c / D];
    const V wv = *reinterpret_cast<const V *>(w + c);
    float *p = dX + r * lddx + c;
    V o;
    if (accumulate) o = *reinterpret_cast<const V *>(p);
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
        const float m = __fmul_rn(gv, reinterpret_cast<const float *>(&wv)[i]);
        reinterpret_cast<float *>(&o)[i] = accumulate ? __fadd_rn(reinterpret_cast<float *>(&o)[i], m) : m;
    }
    *reinterpret_cast<V *>(p) = o;
}

static int attn_vec(int32_t D, std::initializer_list<int64_t> lds, std::initializer_list<const void *> ptrs) {
    for (int v = 4; v > 1; v >>= 1) {
        bool ok = D % v == 0;
        for (int64_t ld : lds) ok = ok && ld % v == 0;
        for (const void *q : ptrs) ok = ok && ((uintptr_t)q % (4 * v)) == 0;
        if (ok) return v;
    }
    return 1;
}

}  // namespace gala

extern "C" int gala_head_attn_f32(int64_t n_rows, int32_t F, int32_t heads, const float *X, int64_t ldx,
                                  const float *w, const float *b, float *out, void *stream) {
    using namespace gala;
    if (n_rows < 0 || F < 1 || heads < 1 || F % heads != 0 || ldx < F) return GALA_ERR_INVALID_ARG;
    if (n_rows == 0) return GALA_OK;
    if (!X || !w || !out) return GALA_ERR_INVALID_ARG;
    const int32_t D = F / heads;
    const int vec = attn_vec(D, {ldx}, {X, w});
    const int64_t total = n_rows * heads;
    hipStream_t hs = (hipStream_t)stream;
    int hw = 1;   // lanes per head: D / vec rounded up to a power of two (D = 47: 64 lanes, 47 live)
    while (hw < D / vec) hw <<= 1;
    if (hw <= 64) {
        const unsigned gb = (unsigned)((total * hw + kBlock - 1) / kBlock);
#define GALA_ATTN_GROUP(V, W) hipLaunchKernelGGL((k_head_attn_group<V, W>), dim3(gb), dim3(kBlock), 0, hs, n_rows, heads, D, X, ldx, w, b, out)
#define GALA_ATTN_HW(V)                                      \
        switch (hw) {                                        \
            case 1: GALA_ATTN_GROUP(V, 1); break;            \
            case 2: GALA_ATTN_GROUP(V, 2); break;            \
            case 4: GALA_ATTN_GROUP(V, 4); break;            \
            case 8: GALA_ATTN_GROUP(V, 8); break;            \
            case 16: GALA_ATTN_GROUP(V, 16); break;          \
            case 32: GALA_ATTN_GROUP(V, 32); break;          \
            default: GALA_ATTN_GROUP(V, 64); break;          \
        }
        if (vec == 4) { GALA_ATTN_HW(4) }
        else if (vec == 2) { GALA_ATTN_HW(2) }
        else { GALA_ATTN_HW(1) }
#undef GALA_ATTN_HW
#undef GALA_ATTN_GROUP
        return launch_status();
    }
    const unsigned blocks = (unsigned)((total + kBlock - 1) / kBlock);
    if (vec == 4) hipLaunchKernelGGL(k_head_attn<4>, dim3(blocks), dim3(kBlock), 0, hs, n_rows, heads, D, X, ldx, w, b, out);
    else if (vec == 2) hipLaunchKernelGGL(k_head_attn<2>, dim3(blocks), dim3(kBlock), 0, hs, n_rows, heads, D, X, ldx, w, b, out);
    else hipLaunchKernelGGL(k_head_attn<1>, dim3(blocks), dim3(kBlock), 0, hs, n_rows, heads, D, X, ldx, w, b, out);
    return launch_status();
}

extern "C" int gala_head_attn_bwd_f32(int64_t n_rows, int32_t F, int32_t heads, const float *g,
                                      const float *w, float *dX, int64_t lddx, int32_t accumulate,
                                      void *stream) {
    using namespace gala;
    if (n_rows < 0 || F < 1 || heads < 1 || F % heads != 0 || lddx < F) return GALA_ERR_INVALID_ARG;
    if (n_rows == 0) return GALA_OK;
    if (!g || !w || !dX) return GALA_ERR_INVALID_ARG;
    const int32_t D = F / heads;
    const int vec = attn_vec(D, {lddx}, {w, dX});
    const int64_t total = n_rows * (F / vec);
    const int64_t blocks = (total + kBlock - 1) / kBlock;
    hipStream_t hs = (hipStream_t)stream;
    if (vec == 4) hipLaunchKernelGGL(k_head_attn_bwd<4>, dim3((unsigned)blocks), dim3(kBlock), 0, hs, n_rows, F, heads, D, g, w, dX, lddx, accumulate);
    else if (vec == 2) hipLaunchKernelGGL(k_head_attn_bwd<2>, dim3((unsigned)blocks), dim3(kBlock), 0, hs, n_rows, F, heads, D, g, w, dX, lddx, accumulate);
    else hipLaunchKernelGGL(k_head_attn_bwd<1>, dim3((unsigned)blocks), dim3(kBlock), 0, hs, n_rows, F, heads, D, g, w, dX, lddx, accumulate);
    return launch_status();
}
