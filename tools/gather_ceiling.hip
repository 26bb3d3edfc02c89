// Random-row gather ceiling on this MI355X (tuning evidence, not product code).
//
// Measures how fast the chip can fetch E uniformly random rows of an [N, F] fp32 table,
// with no ordering constraint: the upper bound for any SpMM on a uniform random graph,
// whose per-edge cost is one X-row fetch.  Compare with k_spmm_rowgroup's time on the
// Products-shaped graph (bench.py / tools/spmm_sweep.py).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/gather_ceiling tools/gather_ceiling.hip
//   tools/gather_ceiling [N] [E] [F]
// With -DGALA_PROBE_LIB -shared -fPIC it builds tools/libgala_probe.so instead, whose
// gala_probe_gather_f32 bench.py times on the benchmark graph's own column array
// (measurement code only; the product library never contains it).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return (uint32_t)x;
}

__global__ void k_fill_idx(int32_t *idx, int64_t E, int32_t N) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < E; t += (int64_t)gridDim.x * blockDim.x)
        idx[t] = (int32_t)(mix(t * 0x9e3779b97f4a7c15ULL + 7) % (uint32_t)N);
}
__global__ void k_fill_x(float *x, int64_t n) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x)
        x[t] = (float)(mix(t) & 1023) * (1.0f / 1024.0f);
}

// A group of G lanes (G*4 floats = one row) walks CHUNK consecutive indices with U rows
// in flight per lane; the group sums its rows (any order) and writes one row.
template <int G, int U, int CHUNK, bool NT>
__global__ __launch_bounds__(256) void k_gather(const int32_t *__restrict__ idx, const float *__restrict__ X,
                                                int64_t E, float *__restrict__ out) {
    const int lane = threadIdx.x & 63, gl = lane & (G - 1);
    const int64_t grp = ((int64_t)blockIdx.x * 256 + threadIdx.x) / G;
    const int64_t e0 = grp * CHUNK;
    if (e0 >= E) return;
    const int64_t e1 = std::min<int64_t>(e0 + CHUNK, E);
    f4 acc = 0.0f;
    for (int64_t e = e0; e < e1; e += U) {
        int32_t c[U];
        f4 x[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int64_t ee = (e + k < e1) ? e + k : e1 - 1;
            c[k] = NT ? __builtin_nontemporal_load(idx + ee) : idx[ee];
        }
#pragma unroll
        for (int k = 0; k < U; ++k) x[k] = *reinterpret_cast<const f4 *>(X + (int64_t)c[k] * (G * 4) + gl * 4);
#pragma unroll
        for (int k = 0; k < U; ++k)
            if (e + k < e1) acc += x[k];
    }
    *reinterpret_cast<f4 *>(out + grp * (G * 4) + gl * 4) = acc;
}

// lds: dynamic LDS per 256-thread workgroup (caps the workgroups per CU: the waves per CU the
// gather gets, e.g. 80 KiB -> 2 workgroups = 8 waves, the input-space GAT kernel's occupancy)
template <int G, int U, int CHUNK, bool NT>
static float run(const int32_t *idx, const float *X, int64_t E, float *out, const char *name, size_t lds = 0) {
    const int64_t groups = (E + CHUNK - 1) / CHUNK;
    const int64_t blocks = (groups * G + 255) / 256;
    if (lds > 65536) CK(hipFuncSetAttribute((const void *)k_gather<G, U, CHUNK, NT>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 2; ++i) hipLaunchKernelGGL((k_gather<G, U, CHUNK, NT>), dim3(blocks), dim3(256), lds, 0, idx, X, E, out);
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < 10; ++r) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((k_gather<G, U, CHUNK, NT>), dim3(blocks), dim3(256), lds, 0, idx, X, E, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const float ms = ts[ts.size() / 2];
    const double row_b = G * 16.0;
    printf("{\"kernel\": \"%s\", \"lds_per_wg\": %zu, \"row_bytes\": %.0f, \"E\": %lld, \"ms\": %.4f, \"rows_per_s\": %.4e, \"row_GBps\": %.1f}\n",
           name, lds, row_b, (long long)E, ms, E / (ms * 1e-3), E * row_b / (ms * 1e-3) / 1e9);
    fflush(stdout);
    return ms;
}

// Unordered gather of X[idx[e], 0:F] for all e (chunks of 64 edges per row group, 4 rows
// in flight per lane), summed per chunk into out[E/64, F].  F = 32, 128 or 256.
extern "C" int gala_probe_gather_f32(const int32_t *idx, const float *X, int64_t E, int32_t F,
                                     float *out, void *stream) {
    constexpr int C = 64;
    const int64_t groups = (E + C - 1) / C;
    hipStream_t st = (hipStream_t)stream;
    if (F == 32)
        hipLaunchKernelGGL((k_gather<8, 4, C, false>), dim3((groups * 8 + 255) / 256), dim3(256), 0, st, idx, X, E, out);
    else if (F == 128)
        hipLaunchKernelGGL((k_gather<32, 8, C, false>), dim3((groups * 32 + 255) / 256), dim3(256), 0, st, idx, X, E, out);
    else if (F == 256)
        hipLaunchKernelGGL((k_gather<64, 4, C, false>), dim3((groups * 64 + 255) / 256), dim3(256), 0, st, idx, X, E, out);
    else
        return -2;
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

#ifndef GALA_PROBE_LIB
int main(int argc, char **argv) {
    const int32_t N = argc > 1 ? atoi(argv[1]) : 2449029;
    const int64_t E = argc > 2 ? atoll(argv[2]) : 126167309LL;
    const int F = argc > 3 ? atoi(argv[3]) : 32;
    int32_t *idx;
    float *X, *out;
    CK(hipMalloc(&idx, E * 4));
    CK(hipMalloc(&X, (int64_t)N * F * 4));
    CK(hipMalloc(&out, (E / 8 + 64) * (int64_t)F * 4));
    hipLaunchKernelGGL(k_fill_idx, dim3(4096), dim3(256), 0, 0, idx, E, N);
    hipLaunchKernelGGL(k_fill_x, dim3(4096), dim3(256), 0, 0, X, (int64_t)N * F);
    CK(hipDeviceSynchronize());
    if (F == 32) {
        run<8, 8, 64, false>(idx, X, E, out, "G8_U8_C64");
        run<8, 16, 64, false>(idx, X, E, out, "G8_U16_C64");
        run<8, 8, 64, true>(idx, X, E, out, "G8_U8_C64_ntidx");
        run<8, 8, 256, false>(idx, X, E, out, "G8_U8_C256");
        run<8, 4, 64, false>(idx, X, E, out, "G8_U4_C64");
    } else if (F == 256) {
        run<64, 4, 64, false>(idx, X, E, out, "G64_U4_C64");
        run<64, 8, 64, false>(idx, X, E, out, "G64_U8_C64");
        run<64, 16, 64, false>(idx, X, E, out, "G64_U16_C64");
    } else if (F == 128) {
        run<32, 8, 64, false>(idx, X, E, out, "G32_U8_C64");
        run<32, 16, 64, false>(idx, X, E, out, "G32_U16_C64");
        // the same gather held to fewer waves per CU (LDS per workgroup of 4 waves)
        for (size_t lds : {20480, 40960, 81920, 160 * 1024}) {
            run<32, 8, 64, false>(idx, X, E, out, "G32_U8_C64_ldscap", lds);
            run<32, 4, 64, false>(idx, X, E, out, "G32_U4_C64_ldscap", lds);
        }
    }
    return 0;
}
#endif
