// diag_kernels.hip — coherence diagnostics (HcclAmdDiagReadByXcc): which XCDs see which bytes of a buffer.
//
// Every workgroup of a 256-workgroup launch (dealt round-robin over the 8 XCDs) reads the whole range and counts the
// 4-byte words that differ from `expect`, and the words that are zero, with plain loads (served by its XCD's L2) or
// non-temporal loads (the executor folds' and the one-sided kernel's load form). Per workgroup it writes
// {mismatches, zeros, XCC id} into out[3 * blockIdx.x ..]. A line one XCD's L2 holds stale shows up on that XCD's
// workgroups only; data still dirty in one XCD's L2 (not yet in memory) shows up on every other XCD.
#include <hip/hip_runtime.h>

#include "comm.h"

namespace hccl_amd {

namespace {

constexpr uint32_t kDiagBlocks = 256;

template <bool NT>
__global__ void __launch_bounds__(256) k_read_by_xcc(const uint32_t* p, const uint32_t* expect, uint64_t words,
                                                     uint32_t* out)
{
    uint32_t bad = 0, zero = 0;
    for (uint64_t i = threadIdx.x; i < words; i += blockDim.x) {
        const uint32_t x = NT ? __builtin_nontemporal_load(p + i) : p[i];
        bad += x != expect[i];
        zero += x == 0;
    }
    __shared__ uint32_t sb, sz;
    if (threadIdx.x == 0) sb = sz = 0;
    __syncthreads();
    atomicAdd(&sb, bad);
    atomicAdd(&sz, zero);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        out[3 * blockIdx.x + 0] = sb;
        out[3 * blockIdx.x + 1] = sz;
        out[3 * blockIdx.x + 2] = xcc & 15u;
    }
}

}  // namespace

}  // namespace hccl_amd

extern "C" HcclResult HcclAmdDiagReadByXcc(const void* p, const void* expect, uint64_t words, int32_t nonTemporal,
                                           void* out, aclrtStream stream)
{
    using namespace hccl_amd;
    if (p == nullptr || expect == nullptr || out == nullptr) return HCCL_E_PTR;
    auto s = static_cast<hipStream_t>(stream);
    const auto* src = static_cast<const uint32_t*>(p);
    const auto* exp = static_cast<const uint32_t*>(expect);
    auto* o = static_cast<uint32_t*>(out);
    if (nonTemporal != 0) {
        hipLaunchKernelGGL(k_read_by_xcc<true>, dim3(kDiagBlocks), dim3(256), 0, s, src, exp, words, o);
    } else {
        hipLaunchKernelGGL(k_read_by_xcc<false>, dim3(kDiagBlocks), dim3(256), 0, s, src, exp, words, o);
    }
    HIP_CHK(hipGetLastError());
    return HCCL_SUCCESS;
}
