// config.h — a communicator's configuration, read from the environment once, when the communicator is created.
//
// The reference reads its environment once per process (InitEnvConfig, src/common/alg_env_config.cc:176) and its
// collectives consult the parsed values. Here every collective consults Comm::cfg; no collective calls getenv (a
// getenv racing a setenv on another thread is undefined behaviour). HcclAmdCommSetConfig changes one entry afterwards
// (tests, the bench's A/B rows).
#pragma once

#include <cstdint>

#include "internal.h"

namespace hccl_amd {

struct CommConfig {
    bool strict = false;                          // HCCL_DETERMINISTIC=strict (alg_env_config.cc:1036-1076)
    bool expansionAiv = false;                    // HCCL_OP_EXPANSION_MODE=AIV
    uint32_t aivCoreLimit = 48;                   // HCCL_AMD_AIV_CORE_LIMIT (MAX_NUM_BLOCKS, aiv_defines.h:35)
    uint64_t singleStreamBytes = 1ull << 20;      // HCCL_AMD_SINGLE_STREAM_BYTES: single-stream programs up to this
    uint64_t smallIpcBytes = 1ull << 20;          // HCCL_AMD_SMALL_IPC_BYTES: AllReduce up to this on the one-sided kernel
    bool planCache = true;                        // HCCL_AMD_PLAN_CACHE
    uint32_t graphCache = 16;                     // HCCL_AMD_GRAPH_CACHE: executor graphs kept (0 = every call eager)
    int32_t ipcLightFence = -1;                   // HCCL_AMD_IPC_LIGHT_FENCE: -1 = per mode (ipc.cc), 0, 1
    bool ipcNt = true;                            // HCCL_AMD_IPC_NT
    uint32_t ipcThreads = 256;                    // HCCL_AMD_IPC_THREADS (256 or 512)
    uint64_t ipcTileBytes = 0;                    // HCCL_AMD_IPC_TILE_KIB (0 = one window per block)
    uint64_t ipcTimeoutMs = 1091000;              // HCCL_AMD_IPC_TIMEOUT_MS, else HCCL_EXEC_TIMEOUT (AIV rule)
    // HCCL_AMD_IPC_STAGING_MIB (read when the one-sided kernel's large staging tier is set up, ipc.h IpcTier): the
    // area size of that tier (four areas per rank); 0 = HCCL_BUFFSIZE / 2, so that the tier holds 2 x HCCL_BUFFSIZE
    // like the reference's CCL buffer pair. Larger areas run large calls in fewer staging rounds (each round costs
    // two barriers and three phase fills and drains: 512 MiB areas were 5-12 % faster than 128 MiB at n = 2 and 4 on
    // C3-sized calls, profiles/r03_ipc_variant_ab_shapes.jsonl); a caller that wants that sets HCCL_BUFFSIZE, as on
    // the reference.
    uint64_t ipcStagingBytes = 0;
    bool ipcTrace = false;                        // HCCL_AMD_IPC_TRACE (diagnostics)
    bool ipcL2Scrub = true;                       // HCCL_AMD_IPC_L2_SCRUB
    bool foldTiming = false;                      // HCCL_AMD_FOLD_TIMING: time the executor's folds (diagnostics)
    uint64_t ipcLlBytes = 64ull << 10;            // HCCL_AMD_IPC_LL_BYTES: one-shot AllReduces up to this many bytes
                                                  // per rank (at most 64 KiB) in the LL form (ipc_kernel_body.h)
    int32_t injectIpcAllocFail = -1;              // HCCL_AMD_INJECT_IPC_ALLOC_FAIL=r (tests): rank r's one-sided
                                                  // set-up allocations fail, as under memory pressure
};

// The configuration a communicator created now takes.
CommConfig ReadCommConfig();
// HcclAmdCommSetConfig / HcclAmdCommGetConfig by HcclAmdConfigKey; HCCL_E_PARA for an unknown key or a value outside
// the key's range.
HcclResult SetConfigEntry(CommConfig& cfg, int32_t key, int64_t value);
HcclResult GetConfigEntry(const CommConfig& cfg, int32_t key, int64_t* value);

}  // namespace hccl_amd
