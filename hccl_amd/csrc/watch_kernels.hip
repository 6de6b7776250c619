// watch_kernels.hip — device side of the execution bound (watchdog.cc).
//
// k_stamp: a collective's start and completion stamps. One lane stores the call's sequence number into the watchdog's
// pinned host ring (a system-scope release store: a vector store, visible to the host's plain loads). A kernel of its
// own costs about 1.8 us of GPU time per stamp on this part, a third of hipStreamWriteValue64's 5.5 us and below an
// event record's 3.0 us (tools/stamp_cost_probe.hip, profiles/r03_stamp_cost.jsonl).
//
// k_stall: the stand-in for a lost peer in the execution-timeout tests (HCCL_AMD_INJECT_STALL_GROUP). One wave waits, as an RCCL receive waits for a message that never comes, until a pinned host word becomes non-zero
// (the watchdog sets it when it aborts the communicator, as ncclCommAbort raises RCCL's abort flag) or until its own
// bound of maxMs has passed, so the kernel always ends. Loads only: system-scope relaxed loads of the coherent word.
#include <hip/hip_runtime.h>

#include "comm.h"

namespace hccl_amd {

namespace {

__global__ void __launch_bounds__(64) k_stall(const uint32_t* word, uint64_t maxTicks)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
    for (;;) {
        if (__hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > maxTicks) break;
        __builtin_amdgcn_s_sleep(127);
    }
}

__global__ void __launch_bounds__(64) k_stamp(uint64_t* slot, uint64_t seq)
{
    if (threadIdx.x == 0) __hip_atomic_store(slot, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

HcclResult LaunchStamp(uint64_t* slot, uint64_t seq, hipStream_t stream)
{
    hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, stream, slot, seq);
    HIP_CHK(hipGetLastError());
    return HCCL_SUCCESS;
}

HcclResult LaunchStall(const uint32_t* word, uint64_t maxMs, hipStream_t stream)
{
    hipLaunchKernelGGL(k_stall, dim3(1), dim3(64), 0, stream, word, maxMs * 100000ull);
    HIP_CHK(hipGetLastError());
    return HCCL_SUCCESS;
}

}  // namespace hccl_amd
