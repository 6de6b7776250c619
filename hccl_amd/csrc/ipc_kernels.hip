// ipc_kernels.hip — dispatch of the one-sided kernels over the per-dtype translation units (ipc_k_*.hip, device
// code in ipc_kernel_body.h) and the L2 maintenance of fresh staging.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>

#include "internal.h"
#include "ipc.h"

namespace hccl_amd {

// Cache maintenance for a fresh staging allocation: every XCD's L2 written back and invalidated at system scope
// (buffer_wbl2 sc0 sc1, buffer_inv sc0 sc1), so that no line a freed buffer left in some L2 is read or written back
// over the new staging. Blocks are dealt round-robin over the XCDs (MI355X_MICROARCH.md, workgroup dispatch): one
// block per CU reaches every L2. Until r01 this was a 512 MiB stream through the cached path (probabilistic eviction,
// ~190 us); the r01 stale-operand failure it was added for no longer reproduces without any maintenance, and the
// barrier's dropped write-back wait (Barrier, ipc_kernel_body.h) is the fault the symptom fits.
__global__ __launch_bounds__(64) void k_l2_maintain()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

HcclResult ScrubL2(hipStream_t stream)
{
    int cus = 256;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) {
        cus = 256;
    }
    hipLaunchKernelGGL(k_l2_maintain, dim3(uint32_t(cus)), dim3(64), 0, stream);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) {
        HCCL_AMD_ERR("L2 maintenance failed: %s", hipGetErrorString(e));
        return HCCL_E_RUNTIME;
    }
    return HCCL_SUCCESS;
}

uint32_t IpcResidentBlocks(HcclDataType dt, HcclReduceOp op, bool rhd, bool ll, uint32_t threads)
{
    // per process and (dtype, op, kind of kernel, block size); one device model per node (0 = not yet asked)
    static std::atomic<uint32_t> cache[32][4][2][2][2];
    const uint32_t di = static_cast<uint32_t>(dt), oi = static_cast<uint32_t>(op), ti = threads > kIpcBlock ? 1 : 0;
    if (di < 32 && oi < 4) {
        const uint32_t v = cache[di][oi][rhd ? 1 : 0][ll ? 1 : 0][ti].load(std::memory_order_relaxed);
        if (v != 0) return v;
    }
    const void* k = nullptr;
    switch (dt) {
        case HCCL_DATA_TYPE_INT8: k = IpcKernel_Int8(op, rhd, ll); break;
        case HCCL_DATA_TYPE_INT16: k = IpcKernel_Int16(op, rhd, ll); break;
        case HCCL_DATA_TYPE_INT32: k = IpcKernel_Int32(op, rhd, ll); break;
        case HCCL_DATA_TYPE_INT64: k = IpcKernel_Int64(op, rhd, ll); break;
        case HCCL_DATA_TYPE_UINT64: k = IpcKernel_Uint64(op, rhd, ll); break;
        case HCCL_DATA_TYPE_FP16: k = IpcKernel_Fp16(op, rhd, ll); break;
        case HCCL_DATA_TYPE_BFP16: k = IpcKernel_Bf16(op, rhd, ll); break;
        case HCCL_DATA_TYPE_FP32: k = IpcKernel_Fp32(op, rhd, ll); break;
        case HCCL_DATA_TYPE_FP64: k = IpcKernel_Fp64(op, rhd, ll); break;
        default: return 0;
    }
    int perCu = 0, cus = 0, dev = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCu, k, static_cast<int>(threads), 0) != hipSuccess ||
        perCu <= 0) {
        return 0;
    }
    // The occupancy API counts VGPRs and LDS but not SGPRs. The hardware admits at most floor(800 / (ceil(sgpr/16)*16
    // + 16)) workgroups of 256 threads per CU (MI355X_MICROARCH.md, "Residency and cooperative launch"): 6 for these
    // kernels' 104-106 SGPRs where the API answered 7 for the fp16 RHD instance, so an 8-rank loopback world asked for
    // 256 blocks per rank waited for blocks that could not start (r03). No kernel of gfx950 allocates more than 112
    // SGPRs, so 6 per CU is always admitted.
    perCu = std::min(perCu, threads > kIpcBlock ? 3 : 6);
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) {
        return 0;
    }
    const uint32_t v = static_cast<uint32_t>(perCu) * static_cast<uint32_t>(cus);
    if (di < 32 && oi < 4) cache[di][oi][rhd ? 1 : 0][ll ? 1 : 0][ti].store(v, std::memory_order_relaxed);
    return v;
}

HcclResult LaunchIpcCollective(const IpcArgs& a, uint32_t blocks, uint32_t worldRanks, HcclDataType dt,
                              HcclReduceOp op, hipStream_t stream)
{
    dim3 grid(blocks, worldRanks == 0 ? 1 : worldRanks);
    hipError_t e;
    switch (dt) {
        case HCCL_DATA_TYPE_INT8: e = LaunchIpc_Int8(op, a, grid, stream); break;
        case HCCL_DATA_TYPE_INT16: e = LaunchIpc_Int16(op, a, grid, stream); break;
        case HCCL_DATA_TYPE_INT32: e = LaunchIpc_Int32(op, a, grid, stream); break;
        case HCCL_DATA_TYPE_INT64: e = LaunchIpc_Int64(op, a, grid, stream); break;
        case HCCL_DATA_TYPE_UINT64: e = LaunchIpc_Uint64(op, a, grid, stream); break;
        case HCCL_DATA_TYPE_FP16: e = LaunchIpc_Fp16(op, a, grid, stream); break;
        case HCCL_DATA_TYPE_BFP16: e = LaunchIpc_Bf16(op, a, grid, stream); break;
        case HCCL_DATA_TYPE_FP32: e = LaunchIpc_Fp32(op, a, grid, stream); break;
        case HCCL_DATA_TYPE_FP64: e = LaunchIpc_Fp64(op, a, grid, stream); break;
        default: return HCCL_E_NOT_SUPPORT;
    }
    if (e != hipSuccess) {
        HCCL_AMD_ERR("ipc collective launch failed: %s", hipGetErrorString(e));
        return HCCL_E_RUNTIME;
    }
    return HCCL_SUCCESS;
}

}  // namespace hccl_amd
