// ipc.h — one-sided AllReduce over peer-mapped staging (host state + kernel launch interface).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/hccl_types.h"

namespace hccl_amd {

constexpr int kIpcMaxRanks = 16;

// Kernel arguments. In rank mode (me >= 0) only in[me] / out[me] are used; stgIn / stgRes / flags hold every rank's
// mapping (own allocation at [me], peers opened through hipIpcOpenMemHandle). In world mode (me < 0) every table is
// full and blockIdx.y is the rank.
struct IpcArgs {
    const void* in[kIpcMaxRanks];
    void* out[kIpcMaxRanks];
    void* stgIn[kIpcMaxRanks];
    void* stgRes[kIpcMaxRanks];
    uint32_t* flags[kIpcMaxRanks];  // [blocks][n] per rank
    uint32_t n;
    int32_t me;
    uint64_t count;
    uint64_t roundElems;
    uint32_t epochBase;
    uint64_t timeoutTicks;  // per barrier wait, in s_memrealtime ticks (100 MHz)
    uint32_t* status;  // [0] bit 0: a barrier timed out (sticky per communicator); [1]: longest wait, in polls
    bool aligned;      // every in[] / out[] the launch touches is 16-B aligned (else element-wise accesses to them)
};

HcclResult LaunchIpcAllReduce(const IpcArgs& a, uint32_t blocks, uint32_t worldRanks, HcclDataType dt,
                              HcclReduceOp op, hipStream_t stream);

// Per-communicator state of the IPC path.
struct IpcState {
    bool ready = false;
    bool unavailable = false;      // set-up failed on some rank: every later call reports NOT_SUPPORT
    void* stg = nullptr;           // own staging: [in area: stgInBytes][result area: stgResBytes], uncached
    uint32_t* flags = nullptr;     // own flags, uncached, zeroed
    uint32_t* status = nullptr;    // device words: [0] bit 0 = barrier timeout, [1] = longest barrier wait (polls)
    void* peerStg[kIpcMaxRanks] = {};
    uint32_t* peerFlags[kIpcMaxRanks] = {};
    bool opened[kIpcMaxRanks] = {};
    uint64_t stgInBytes = 0;
    uint64_t stgResBytes = 0;
    uint32_t epoch = 0;
    uint32_t blocks = 0;
};

constexpr uint32_t kIpcBlocks = 128;
constexpr size_t kIpcStatusBytes = 16;  // status words, reset as one 16-B block per call
constexpr uint64_t kIpcStagingBytes = 128ull << 20;  // slot area per rank; the result area is as large

}  // namespace hccl_amd
