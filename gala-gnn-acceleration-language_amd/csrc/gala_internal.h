// Internal helpers shared by the gfx950 kernels of libgala_hip.so.
//
// Numerics contract: the library is compiled with -ffp-contract=off and every rounding
// step is written out (fmaf where nvcc contracts the reference's `a + b*c`, __fmul_rn /
// __fadd_rn elsewhere), so that a kernel that keeps the reference's per-row edge order
// is bit-identical to the reference kernel (src/codegen/cuda.h:286-436).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gala_hip.h"

namespace gala {

constexpr int kWave = 64;          // CDNA wavefront
constexpr int kBlock = 256;        // 4 waves per workgroup
constexpr int kXcds = 8;           // MI355X: 8 XCDs, each with its own 4 MB L2

// XCD-aware block order.  The dispatcher sends workgroup b to XCD b % 8, so consecutive
// blocks -- neighbouring rows -- land on different XCDs and the neighbour rows they share
// are fetched into eight L2s.  logical_block_runs() hands every XCD runs of K consecutive
// logical blocks, the XCDs interleaved run by run, so all XCDs stay in the same region of
// the graph (shared Infinity Cache, balanced load) while rows that share neighbours share
// an L2.  A bijection on [0, nb): the tail past the last full round keeps its order.
// Measured on Products-shaped graphs (profiles/r01_xcd_order_ab.jsonl: xcd 0 = hardware
// order, 1 = one contiguous range per XCD, 16 / 64 = runs of K; K = 64): banded graphs with
// neighbours within +-2048 rows 1.41 -> 1.27 ms at F = 32, uniform 2.44 -> 2.41 ms, no
// case more than ~1 % slower; one contiguous range per XCD instead lost up to 28 %.
constexpr int64_t kXcdRun = 64;
__device__ __forceinline__ int64_t logical_block_runs(int64_t b, int64_t nb, int64_t K) {
    const int64_t full = nb - nb % (kXcds * K);
    if (b >= full) return b;
    const int64_t x = b % kXcds, i = b / kXcds;
    return ((i / K) * kXcds + x) * K + i % K;
}
constexpr int kMaxSegPerLaunch = 64;

// Segment table passed by value (kernel arguments live in the scalar cache).
struct SegTable {
    int32_t n;                         // segments in this launch
    int32_t base[kMaxSegPerLaunch];    // first edge of each segment (seg_bounds[2s])
    int32_t rp[kMaxSegPerLaunch];      // index of the segment's rowptr block (s)
};

// Kernel-argument structs keep the segment table by value; indexing it with a runtime
// segment id must not copy the array into VGPRs, so kernels read it through the kernarg
// segment pointer (scalar loads).  `off` = offsetof(<params struct>, seg); the params
// struct is the kernel's first argument (kernarg offset 0).
typedef const SegTable __attribute__((address_space(4))) *KernargSegPtr;
__device__ __forceinline__ KernargSegPtr kernarg_segtable(size_t off) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const char __attribute__((address_space(4))) *KernargBytes;
    return (KernargSegPtr)((KernargBytes)__builtin_amdgcn_kernarg_segment_ptr() + off);
#else
    (void)off;
    return nullptr;
#endif
}

// Thread-local last HIP error (the only mutable state of the library).
void set_last_hip_error(int e);

int check_csr(const gala_csr_t *A);
int fill_segments(const gala_csr_t *A, int32_t first, SegTable *t);
int launch_status();  // hipGetLastError -> gala_status

__device__ __forceinline__ float ld_nt(const float *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ int32_t ld_nt(const int32_t *p) { return __builtin_nontemporal_load(p); }

// Wave-uniform value broadcast (keeps the row bounds in SGPRs).
__device__ __forceinline__ int32_t uniform(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Lane i's partner i ^ O.  O <= 8 stays inside a 16-lane DPP row: a VALU data-parallel move
// (quad_perm for 1 and 2; for 4 and 8 a row shift each way, picked by the lane's bit), where
// __shfl_xor is a ds_bpermute through the LDS crossbar whose result the next step must wait
// for.  Every lane of the row must be active.  row_shl:n reads lane i + n, row_shr:n lane i - n.
template <int O>
__device__ __forceinline__ float lane_xor(float v) {
    const int x = __float_as_int(v);
    if constexpr (O == 1) {
        return __int_as_float(__builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, true));  // quad_perm [1,0,3,2]
    } else if constexpr (O == 2) {
        return __int_as_float(__builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, true));  // quad_perm [2,3,0,1]
    } else if constexpr (O == 4 || O == 8) {
        const int up = __builtin_amdgcn_mov_dpp(x, 0x100 + O, 0xF, 0xF, true);    // row_shl:O
        const int down = __builtin_amdgcn_mov_dpp(x, 0x110 + O, 0xF, 0xF, true);  // row_shr:O
        return __int_as_float((threadIdx.x & O) ? down : up);
    } else {
        return __shfl_xor(v, O, 64);
    }
}

// xor-butterfly inside aligned groups of W lanes (W power of two <= 64): partners W/2, ..., 1,
// each step v + partner (every lane ends with the same bits).  Partners below 16 are DPP moves
// (lane_xor); all lanes of a group must be active.
template <int W>
__device__ __forceinline__ float group_sum(float v) {
    if constexpr (W >= 2) {
        v += lane_xor<W / 2>(v);
        return group_sum<W / 2>(v);
    } else {
        return v;
    }
}
template <int W>
__device__ __forceinline__ float group_max(float v) {
    if constexpr (W >= 2) {
        v = fmaxf(v, lane_xor<W / 2>(v));
        return group_max<W / 2>(v);
    } else {
        return v;
    }
}

}  // namespace gala
