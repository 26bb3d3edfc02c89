// Measurement probe: which compute units a CU-masked stream's workgroups run on
// (hipExtStreamCreateWithCUMask).  Every workgroup's lane 0 stores its hardware ids
// (HW_ID: CU / SH / SE, XCC_ID) with a vector store; the host prints the distinct
// (xcc, se, sh, cu) set each mask reached.  The masks keep at least one CU of every XCD
// under either bit order (bits 0-7 and every 32nd bit), so every workgroup has a CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <set>
#include <tuple>
#include <vector>

__global__ void k_where(unsigned *out) {
    if (threadIdx.x == 0) {
        unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_REG_HW_ID, 32 bits
        unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
        out[2 * blockIdx.x] = hw;
        out[2 * blockIdx.x + 1] = xcc;
        // keep the workgroup resident a little, so many CUs are used
        long long t0 = wall_clock64();
        while (wall_clock64() - t0 < 2000) {}
    }
}

static void run(const char *name, const std::vector<unsigned> &mask) {
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, (unsigned)mask.size(), mask.data()) != hipSuccess) {
        printf("%s: hipExtStreamCreateWithCUMask failed\n", name);
        return;
    }
    const int nb = 4096;
    unsigned *d;
    hipMalloc(&d, nb * 2 * sizeof(unsigned));
    hipLaunchKernelGGL(k_where, dim3(nb), dim3(64), 0, s, d);
    hipError_t e = hipStreamSynchronize(s);
    std::vector<unsigned> h(nb * 2);
    hipMemcpy(h.data(), d, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost);
    std::set<std::tuple<unsigned, unsigned, unsigned, unsigned>> cus;
    std::set<unsigned> xccs;
    for (int b = 0; b < nb; ++b) {
        unsigned hw = h[2 * b], xcc = h[2 * b + 1] & 0xf;
        unsigned cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x7;
        cus.insert({xcc, se, sh, cu});
        xccs.insert(xcc);
    }
    printf("%s: rc=%d distinct CUs %zu, XCCs %zu:", name, (int)e, cus.size(), xccs.size());
    for (auto &c : cus) printf(" (%u,%u,%u,%u)", std::get<0>(c), std::get<1>(c), std::get<2>(c), std::get<3>(c));
    printf("\n");
    hipFree(d);
    hipStreamDestroy(s);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    printf("multiProcessorCount %d\n", p.multiProcessorCount);
    const int words = (p.multiProcessorCount + 31) / 32;
    std::vector<unsigned> all(words, 0xffffffffu), low8(words, 0), every32(words, 0), both(words, 0), rest(words, 0);
    low8[0] = 0xff;
    for (int w = 0; w < words; ++w) every32[w] = 1u;
    for (int w = 0; w < words; ++w) both[w] = low8[w] | every32[w];
    for (int w = 0; w < words; ++w) rest[w] = ~both[w];
    run("all", all);
    run("bits0-7+every32nd", both);
    run("complement", rest);
    return 0;
}
