// internal.h — shared declarations of libhccl_amd.so (not installed; the public ABI is include/*.h).
#pragma once

#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "../../include/hccl.h"
#include "../../include/hccl_amd.h"

namespace hccl_amd {

// ---- host profile (executor.cc; HCCL_AMD_HOST_PROFILE=1, read once): host time per HCCL_AMD_HP_* category,
// reported by HcclAmdHostProfile.
bool HostProfileOn();
void HostProfileAdd(int cat, uint64_t ns);

class HostProfileScope {
public:
    explicit HostProfileScope(int cat) : cat_(HostProfileOn() ? cat : -1)
    {
        if (cat_ >= 0) t0_ = std::chrono::steady_clock::now();
    }
    ~HostProfileScope()
    {
        if (cat_ < 0) return;
        const auto d = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0_);
        HostProfileAdd(cat_, static_cast<uint64_t>(d.count()));
    }
    HostProfileScope(const HostProfileScope&) = delete;
    HostProfileScope& operator=(const HostProfileScope&) = delete;

private:
    int cat_;
    std::chrono::steady_clock::time_point t0_;
};

// Reduce ops in the same numbering as HcclReduceOp.
enum ROp : int { R_SUM = 0, R_PROD = 1, R_MAX = 2, R_MIN = 3 };

// Element size of each HcclDataType (alg_param.h:43-61 DATATYPE_SIZE_TABLE); 0 = unknown.
uint32_t DataTypeSize(HcclDataType dt);

// True for the dtypes the reduce ops accept (op_common.cc:2913-2957 CheckDataType(needReduce=true)).
bool IsReduceDataType(HcclDataType dt);

// ---- streaming reduce kernels (reduce_kernels.hip)
// out = src (op) dst, element-wise.
HcclResult LaunchReduce2(void* out, const void* src, const void* dst, uint64_t count, HcclDataType dt,
                         HcclReduceOp op, hipStream_t stream);
// out = fold(srcs[0..n)) with acc = srcs[j] (op) acc.
HcclResult LaunchReduceN(void* out, const void* const* srcs, uint32_t n, uint64_t count, HcclDataType dt,
                         HcclReduceOp op, hipStream_t stream);
HcclResult SetReduceLaunch(uint32_t blocksPerCu, uint32_t unroll, uint32_t cachePolicy);
HcclResult SetFoldMode(uint32_t mode);

// Several independent ordered folds with the same operand count in ONE launch (blockIdx.y = segment): the executor
// batches the consecutive REDUCE records of a schedule step (a MeshChunk piece's O6 sub-slices, the R rings' or RHD
// instances' folds). Segments must not overlap each other's outputs. Falls back to one launch per segment when a
// segment's pointers do not share a 16-B phase.
constexpr uint32_t kMaxBatchSegs = 8;
struct FoldSeg {
    void* out;
    const void* srcs[HCCL_AMD_IR_MAX_SRC];
    uint64_t count;
};
HcclResult LaunchReduceNBatch(const FoldSeg* segs, uint32_t nseg, uint32_t nsrc, HcclDataType dt, HcclReduceOp op,
                              hipStream_t stream);

// dst = src over `bytes` bytes on `stream`: every device-to-device copy the library makes is this copy kernel, never
// hipMemcpyAsync (r04: the runtime copy's writes showed up late in the r03 order; DESIGN.md §5b, device copies).
HcclResult LaunchCopyBytes(void* dst, const void* src, uint64_t bytes, hipStream_t stream);

// HCCL_EXEC_TIMEOUT in the reference's format (ParseExecTimeout, alg_env_config.cc:75-110): false when unset or
// malformed, else *seconds (>= 0, <= UINT32_MAX, at most two decimals).
bool ParseExecTimeoutSeconds(const char* env, double* seconds);
// Barrier wait bound of the IPC kernel in s_memrealtime ticks (100 MHz); ipc.cc.
uint64_t IpcTimeoutTicks();

// ---- logging
bool DebugEnabled();

}  // namespace hccl_amd

#define HCCL_AMD_LOG(fmt, ...)                                                                   \
    do {                                                                                         \
        if (hccl_amd::DebugEnabled()) {                                                          \
            std::fprintf(stderr, "[hccl_amd] %s:%d " fmt "\n", __FILE__, __LINE__, ##__VA_ARGS__); \
        }                                                                                        \
    } while (0)

#define HCCL_AMD_ERR(fmt, ...) std::fprintf(stderr, "[hccl_amd][ERROR] %s:%d " fmt "\n", __FILE__, __LINE__, ##__VA_ARGS__)

#define HIP_CHK(expr)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess) {                                                            \
            HCCL_AMD_ERR("%s failed: %s", #expr, hipGetErrorString(e_));                   \
            return HCCL_E_RUNTIME;                                                         \
        }                                                                                  \
    } while (0)

#define HCCL_CHK(expr)                     \
    do {                                   \
        HcclResult r_ = (expr);            \
        if (r_ != HCCL_SUCCESS) return r_; \
    } while (0)
