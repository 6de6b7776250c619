// ipc.h — one-sided AllReduce / ReduceScatter / Reduce over peer-mapped staging (host state + launch interface).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/hccl_types.h"

namespace hccl_amd {

constexpr int kIpcMaxRanks = 16;

enum IpcKind : uint32_t {
    kIpcAllReduce = 0,      // order O2 (acc = x_0, then x_1 .. x_{n-1}); every rank gets every chunk
    kIpcReduceScatter = 1,  // order O1 per block owner (x_me first, then ascending); rank c gets block c
    kIpcReduce = 2,         // order O1 with the chunk owner first (two-shot Reduce); only the root gets the result
};

// Kernel arguments. In rank mode (me >= 0) only in[me] / out[me] are used; stgIn / stgRes / flags hold every rank's
// mapping (own allocation at [me], peers opened through hipIpcOpenMemHandle). In world mode (me < 0) every table is
// full and blockIdx.y is the rank.
//
// Geometry (elements): chunk c of the input starts at c * chunkStride and holds min(chunkLen, total - c*chunkStride)
// elements (clamped at 0), or, balanced (the two-shot Reduce's split), starts at c*chunkLen + min(c, rem) and holds
// chunkLen + (c < rem); rank c owns chunk c. Round k handles piece k of every chunk: chunk elements
// [k*piece, (k+1)*piece). Block b always handles piece coordinates [b*blockElems, (b+1)*blockElems), so every round
// of a launch touches the same slot and result addresses per block and the per-block barrier is sound.
// Staging: owner c's slot q = stgIn[c] + q*piece; results of chunk c at stgRes[p] + c*piece.
struct IpcArgs {
    const void* in[kIpcMaxRanks];
    void* out[kIpcMaxRanks];
    void* stgIn[kIpcMaxRanks];
    void* stgRes[kIpcMaxRanks];
    uint32_t* flags[kIpcMaxRanks];  // [blocks][n] per rank
    uint32_t n;
    int32_t me;
    uint32_t kind;  // IpcKind
    uint32_t root;  // kIpcReduce
    uint64_t total;
    uint64_t chunkStride;
    uint64_t chunkLen;
    uint64_t rem;   // balanced: chunk c starts at c*chunkLen + min(c, rem) and holds chunkLen + (c < rem) elements
    bool balanced;
    uint64_t piece;
    uint64_t blockElems;
    uint32_t rounds;
    uint32_t epochBase;
    uint64_t timeoutTicks;  // per barrier wait, in s_memrealtime ticks (100 MHz)
    uint32_t* status;  // [0] bit 0: a barrier timed out (sticky per communicator); [1]: longest wait, in polls
    bool aligned;      // every in[] / out[] is 16-B aligned (chunks whose start is not are still element-wise)
};

HcclResult LaunchIpcCollective(const IpcArgs& a, uint32_t blocks, uint32_t worldRanks, HcclDataType dt,
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
