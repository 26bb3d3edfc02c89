// chain_probe.hip -- what one dependent fp32 add chain costs per element on gfx950, the
// bound of the REF-order hub kernel (k_spmm_hub_exact's chain wave).
//   reg            acc = acc + r[k] over values held in registers (the latency floor)
//   lds_ahead2     the hub chain's loop: 16-B LDS reads of an edge quad, issued two 16-edge
//                  groups ahead of the adds (as in spmm.hip's run_chain)
//   lds_ahead1     the same with one group ahead
//   lds_interleaved one 16-B read between every four adds, 8 quads ahead
//   lanes < 64     the same loop with only that many lanes of the wave active (the others exit)
//   lds_b64_ahead2 8-B reads of an edge pair, 8 reads per 16-edge group
//   row4 / row2    a lane owns 4 (2) features: one 16-B (8-B) read per edge of the lane's
//                  features, 4 (2) independent chains, reads two 8-edge groups ahead; per edge
//                  the chains advance one add each (ns_per_add is then per edge)
//   reg4           the floor of that: 4 chains over registers
// One workgroup of 64 lanes (one wave), n adds per lane; cycles from s_memtime around the
// loop (shader clock), time from HIP events.  Measurement only.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/chain_probe tools/chain_probe.hip && tools/chain_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float F4 __attribute__((ext_vector_type(4)));
typedef float F2 __attribute__((ext_vector_type(2)));

enum Mode { REG, AHEAD2, AHEAD1, INTERLEAVED, B64, ROW4, ROW2, REG4 };

template <int MODE, int LANES>
__global__ __launch_bounds__(64) void k_chain(const float *seed, float *out, long long *cycles, int n) {
    __shared__ F4 buf[1024];  // 16 KB: lane l reads the 16 B at buf[q * 16 + l % 16]
    const int lane = threadIdx.x;
    for (int i = lane; i < 1024; i += 64) {
        const float s = seed[i % 64];
        buf[i] = F4{s, s * 0.5f, s * 0.25f, s * 0.125f};
    }
    __syncthreads();
    if (lane >= LANES) return;
    float r[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) r[k] = seed[(lane + k) % 64] * 1e-3f;
    float acc = 0.0f;
    const long long t0 = __builtin_amdgcn_s_memtime();
    // the clock read (a scalar memory op, returned out of order with LDS reads) completes
    // here: pending, it would make every LDS wait in the loops below a full lgkmcnt(0)
    __builtin_amdgcn_s_waitcnt(0xc07f);
    if constexpr (MODE == INTERLEAVED) {
        constexpr int D = 8;
        const F4 *b = buf + (lane & 15);
        F4 g[D];
#pragma unroll
        for (int k = 0; k < D; ++k) {
            g[k] = b[(k & 63) * 16];
            __builtin_amdgcn_sched_barrier(0);
        }
        for (int i = 0, q = 0; i < n; i += 4 * D, q += D) {
#pragma unroll
            for (int k = 0; k < D; ++k) {
#pragma unroll
                for (int v = 0; v < 4; ++v) acc = __fadd_rn(acc, g[k][v]);
                g[k] = b[((q + D + k) & 63) * 16];
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    } else if constexpr (MODE == REG4) {
        float a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
        for (int i = 0; i < n; i += 16) {
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                acc = __fadd_rn(acc, r[k]);
                a1 = __fadd_rn(a1, r[(k + 1) & 15]);
                a2 = __fadd_rn(a2, r[(k + 2) & 15]);
                a3 = __fadd_rn(a3, r[(k + 3) & 15]);
            }
        }
        acc += a1 + a2 + a3;
    } else if constexpr (MODE == ROW4 || MODE == ROW2) {
        constexpr int NV = MODE == ROW4 ? 4 : 2;
        typedef float VT __attribute__((ext_vector_type(NV)));
        constexpr int GE = 8;  // edges per group
        const VT *b = reinterpret_cast<const VT *>(buf) + (lane & 15);
        constexpr int WRAP = 1024 * 4 / NV / 16;  // edges in the buffer
        VT g[3][GE];
        float a[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) a[v] = 0.0f;
        int q = 0;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
#pragma unroll
            for (int u = 0; u < GE; ++u) g[s][u] = b[((q + u) % WRAP) * 16];
            q += GE;
        }
        for (int i = 0; i < n; i += 3 * GE) {
#pragma unroll
            for (int s = 0; s < 3; ++s) {
                const int nx = (s + 2) % 3;
#pragma unroll
                for (int u = 0; u < GE; ++u) g[nx][u] = b[((q + u) % WRAP) * 16];
                q += GE;
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < GE; ++u)
#pragma unroll
                    for (int v = 0; v < NV; ++v) a[v] = __fadd_rn(a[v], g[s][u][v]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int v = 0; v < NV; ++v) acc += a[v];
    } else if constexpr (MODE == REG) {
        for (int i = 0; i < n; i += 16) {
#pragma unroll
            for (int k = 0; k < 16; ++k) acc = __fadd_rn(acc, r[k]);
        }
    } else if constexpr (MODE == B64) {
        // edge pairs: 8 reads of 8 B per 16-edge group, two groups ahead
        const F2 *b = reinterpret_cast<const F2 *>(buf) + 2 * (lane & 15);
        F2 g[3][8];
        int q = 0;
#pragma unroll
        for (int a = 0; a < 2; ++a) {
#pragma unroll
            for (int u = 0; u < 8; ++u) g[a][u] = b[((q + u) & 127) * 32];
            q += 8;
        }
        for (int i = 0; i < n; i += 48) {
#pragma unroll
            for (int s = 0; s < 3; ++s) {
                const int nx = (s + 2) % 3;
#pragma unroll
                for (int u = 0; u < 8; ++u) g[nx][u] = b[((q + u) & 127) * 32];
                q += 8;
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < 8; ++u)
#pragma unroll
                    for (int v = 0; v < 2; ++v) acc = __fadd_rn(acc, g[s][u][v]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    } else {
        // quads of 4 edges: 4 reads per 16-edge group, AHEAD groups in flight
        constexpr int AHEAD = MODE == AHEAD2 ? 2 : 1;
        const F4 *b = buf + (lane & 15);
        F4 g[AHEAD + 1][4];
        int q = 0;
#pragma unroll
        for (int a = 0; a < AHEAD; ++a) {
#pragma unroll
            for (int u = 0; u < 4; ++u) g[a][u] = b[((q + u) & 63) * 16];
            q += 4;
        }
        for (int i = 0; i < n; i += 16 * (AHEAD + 1)) {
#pragma unroll
            for (int s = 0; s <= AHEAD; ++s) {
                const int nx = (s + AHEAD) % (AHEAD + 1);
#pragma unroll
                for (int u = 0; u < 4; ++u) g[nx][u] = b[((q + u) & 63) * 16];
                q += 4;
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int v = 0; v < 4; ++v) acc = __fadd_rn(acc, g[s][u][v]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[lane] = acc;
    if (lane == 0) cycles[0] = t1 - t0;
}

template <int MODE, int LANES = 64>
static void run(const char *name, const float *seed, float *out, long long *cyc, int n) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL((k_chain<MODE, LANES>), dim3(1), dim3(64), 0, 0, seed, out, cyc, n);  // warm
    (void)hipEventRecord(a);
    hipLaunchKernelGGL((k_chain<MODE, LANES>), dim3(1), dim3(64), 0, 0, seed, out, cyc, n);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    long long c = 0;
    (void)hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("{\"mode\": \"%s\", \"lanes\": %d, \"adds\": %d, \"ms\": %.4f, \"ns_per_add\": %.3f, "
           "\"memtime_ticks_per_add\": %.3f}\n",
           name, LANES, n, ms, ms * 1e6 / n, (double)c / n);
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 388128;  // a multiple of 48
    float *seed, *out;
    long long *cyc;
    (void)hipMalloc(&seed, 64 * sizeof(float));
    (void)hipMalloc(&out, 64 * sizeof(float));
    (void)hipMalloc(&cyc, sizeof(long long));
    float h[64];
    for (int i = 0; i < 64; ++i) h[i] = 0.001f * (i + 1);
    (void)hipMemcpy(seed, h, sizeof(h), hipMemcpyHostToDevice);
    run<REG>("reg", seed, out, cyc, n);
    run<AHEAD2>("lds_ahead2", seed, out, cyc, n);
    run<AHEAD1>("lds_ahead1", seed, out, cyc, n);
    run<INTERLEAVED>("lds_interleaved", seed, out, cyc, n);
    run<AHEAD2, 32>("lds_ahead2", seed, out, cyc, n);
    run<AHEAD2, 16>("lds_ahead2", seed, out, cyc, n);
    run<AHEAD2, 4>("lds_ahead2", seed, out, cyc, n);
    run<B64>("lds_b64_ahead2", seed, out, cyc, n);
    run<REG, 16>("reg", seed, out, cyc, n);
    run<REG4>("reg4", seed, out, cyc, n);
    run<ROW4>("row4", seed, out, cyc, n);
    run<ROW4, 8>("row4", seed, out, cyc, n);
    run<ROW2>("row2", seed, out, cyc, n);
    run<ROW2, 16>("row2", seed, out, cyc, n);
    return 0;
}
