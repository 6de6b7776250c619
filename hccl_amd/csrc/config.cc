// config.cc — the environment, read once per communicator (config.h).
#include "config.h"
#include "ipc.h"

#include <strings.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace hccl_amd {

namespace {

const char* Env(const char* name)
{
    const char* e = std::getenv(name);
    return (e != nullptr && *e != '\0') ? e : nullptr;
}

bool EnvIs(const char* name, const char* value, bool dflt)
{
    const char* e = Env(name);
    return e == nullptr ? dflt : std::strcmp(e, value) == 0;
}

bool EnvU64(const char* name, uint64_t* out)
{
    const char* e = Env(name);
    if (e == nullptr) return false;
    char* end = nullptr;
    const unsigned long long v = std::strtoull(e, &end, 10);
    if (end == e) return false;
    *out = v;
    return true;
}

// The barrier wait bound of the one-sided kernel. It is the reference's AIV engine, so HCCL_EXEC_TIMEOUT follows its
// AIV-mode rule (docs/zh/user_guide/hccl_env/HCCL_EXEC_TIMEOUT.md): seconds with at most two decimals, default 1091,
// and 0 or anything above 1091 taken as 1091. A malformed value is ignored with the default, as ParseExecTimeout does
// (src/common/alg_env_config.cc:75-110). HCCL_AMD_IPC_TIMEOUT_MS (1 ms .. 1 h), when set, takes precedence: it is the
// tests' and the benchmark's short bound.
uint64_t IpcTimeoutMsFromEnv()
{
    uint64_t v = 0;
    if (EnvU64("HCCL_AMD_IPC_TIMEOUT_MS", &v) && v >= 1 && v <= 3600000ull) return v;
    constexpr uint64_t kAivMaxMs = 1091000;
    double sec = 0;
    if (ParseExecTimeoutSeconds(std::getenv("HCCL_EXEC_TIMEOUT"), &sec) && sec > 0) {
        const double m = sec * 1000.0;
        return m >= double(kAivMaxMs) ? kAivMaxMs : std::max<uint64_t>(1, static_cast<uint64_t>(m + 0.5));
    }
    return kAivMaxMs;
}

}  // namespace

CommConfig ReadCommConfig()
{
    CommConfig c;
    const char* det = Env("HCCL_DETERMINISTIC");
    c.strict = det != nullptr && strcasecmp(det, "strict") == 0;
    c.expansionAiv = EnvIs("HCCL_OP_EXPANSION_MODE", "AIV", false);
    uint64_t v = 0;
    if (EnvU64("HCCL_AMD_AIV_CORE_LIMIT", &v) && v >= 1 && v <= 4096) c.aivCoreLimit = static_cast<uint32_t>(v);
    if (EnvU64("HCCL_AMD_SINGLE_STREAM_BYTES", &v)) c.singleStreamBytes = v;
    if (EnvU64("HCCL_AMD_SMALL_IPC_BYTES", &v)) c.smallIpcBytes = v;
    c.planCache = !EnvIs("HCCL_AMD_PLAN_CACHE", "0", false);
    if (EnvU64("HCCL_AMD_GRAPH_CACHE", &v)) c.graphCache = static_cast<uint32_t>(std::min<uint64_t>(v, 1024));
    if (const char* f = Env("HCCL_AMD_IPC_LIGHT_FENCE")) c.ipcLightFence = std::strcmp(f, "0") != 0 ? 1 : 0;
    c.ipcNt = !EnvIs("HCCL_AMD_IPC_NT", "0", false);
    c.ipcThreads = EnvIs("HCCL_AMD_IPC_THREADS", "512", false) ? 512u : 256u;
    if (EnvU64("HCCL_AMD_IPC_TILE_KIB", &v) && v <= (1u << 20)) c.ipcTileBytes = v << 10;  // the setter's range
    c.ipcTimeoutMs = IpcTimeoutMsFromEnv();
    // the staging allocation stays below 2 GiB (ipc.cc IpcSetupTier): areas of 16 .. 1000 MiB
    if (EnvU64("HCCL_AMD_IPC_STAGING_MIB", &v) && v >= 16 && v <= 1000) c.ipcStagingBytes = v << 20;
    c.ipcTrace = EnvIs("HCCL_AMD_IPC_TRACE", "1", false);
    c.ipcL2Scrub = !EnvIs("HCCL_AMD_IPC_L2_SCRUB", "0", false);
    c.foldTiming = EnvIs("HCCL_AMD_FOLD_TIMING", "1", false);
    if (EnvU64("HCCL_AMD_IPC_LL_BYTES", &v) && v <= kIpcLlMaxBytes) c.ipcLlBytes = v;
    if (EnvU64("HCCL_AMD_INJECT_IPC_ALLOC_FAIL", &v) && v < (1u << 20)) c.injectIpcAllocFail = static_cast<int32_t>(v);
    return c;
}

HcclResult SetConfigEntry(CommConfig& c, int32_t key, int64_t value)
{
    const auto in = [value](int64_t lo, int64_t hi) { return value >= lo && value <= hi; };
    const auto flag = [&]() { return in(0, 1); };
    switch (key) {
        case HCCL_AMD_CFG_DETERMINISTIC_STRICT: if (!flag()) return HCCL_E_PARA; c.strict = value != 0; break;
        case HCCL_AMD_CFG_EXPANSION_MODE_AIV: if (!flag()) return HCCL_E_PARA; c.expansionAiv = value != 0; break;
        case HCCL_AMD_CFG_AIV_CORE_LIMIT:
            if (!in(1, 4096)) return HCCL_E_PARA;
            c.aivCoreLimit = static_cast<uint32_t>(value);
            break;
        case HCCL_AMD_CFG_SINGLE_STREAM_BYTES:
            if (value < 0) return HCCL_E_PARA;
            c.singleStreamBytes = static_cast<uint64_t>(value);
            break;
        case HCCL_AMD_CFG_SMALL_IPC_BYTES:
            if (value < 0) return HCCL_E_PARA;
            c.smallIpcBytes = static_cast<uint64_t>(value);
            break;
        case HCCL_AMD_CFG_PLAN_CACHE: if (!flag()) return HCCL_E_PARA; c.planCache = value != 0; break;
        case HCCL_AMD_CFG_GRAPH_CACHE:
            if (!in(0, 1024)) return HCCL_E_PARA;
            c.graphCache = static_cast<uint32_t>(value);
            break;
        case HCCL_AMD_CFG_IPC_LIGHT_FENCE:
            if (!in(-1, 1)) return HCCL_E_PARA;
            c.ipcLightFence = static_cast<int32_t>(value);
            break;
        case HCCL_AMD_CFG_IPC_NT: if (!flag()) return HCCL_E_PARA; c.ipcNt = value != 0; break;
        case HCCL_AMD_CFG_IPC_THREADS:
            if (value != 256 && value != 512) return HCCL_E_PARA;
            c.ipcThreads = static_cast<uint32_t>(value);
            break;
        case HCCL_AMD_CFG_IPC_TILE_KIB:
            if (!in(0, 1 << 20)) return HCCL_E_PARA;
            c.ipcTileBytes = static_cast<uint64_t>(value) << 10;
            break;
        case HCCL_AMD_CFG_IPC_TIMEOUT_MS:
            if (!in(1, 3600000)) return HCCL_E_PARA;
            c.ipcTimeoutMs = static_cast<uint64_t>(value);
            break;
        case HCCL_AMD_CFG_IPC_STAGING_MIB:
            if (value != 0 && !in(16, 1000)) return HCCL_E_PARA;
            c.ipcStagingBytes = static_cast<uint64_t>(value) << 20;
            break;
        case HCCL_AMD_CFG_IPC_TRACE: if (!flag()) return HCCL_E_PARA; c.ipcTrace = value != 0; break;
        case HCCL_AMD_CFG_IPC_L2_SCRUB: if (!flag()) return HCCL_E_PARA; c.ipcL2Scrub = value != 0; break;
        case HCCL_AMD_CFG_FOLD_TIMING: if (!flag()) return HCCL_E_PARA; c.foldTiming = value != 0; break;
        case HCCL_AMD_CFG_IPC_LL_BYTES:
            if (!in(0, int64_t(kIpcLlMaxBytes))) return HCCL_E_PARA;
            c.ipcLlBytes = static_cast<uint64_t>(value);
            break;
        default: return HCCL_E_PARA;
    }
    return HCCL_SUCCESS;
}

HcclResult GetConfigEntry(const CommConfig& c, int32_t key, int64_t* value)
{
    switch (key) {
        case HCCL_AMD_CFG_DETERMINISTIC_STRICT: *value = c.strict; break;
        case HCCL_AMD_CFG_EXPANSION_MODE_AIV: *value = c.expansionAiv; break;
        case HCCL_AMD_CFG_AIV_CORE_LIMIT: *value = c.aivCoreLimit; break;
        case HCCL_AMD_CFG_SINGLE_STREAM_BYTES: *value = static_cast<int64_t>(c.singleStreamBytes); break;
        case HCCL_AMD_CFG_SMALL_IPC_BYTES: *value = static_cast<int64_t>(c.smallIpcBytes); break;
        case HCCL_AMD_CFG_PLAN_CACHE: *value = c.planCache; break;
        case HCCL_AMD_CFG_GRAPH_CACHE: *value = c.graphCache; break;
        case HCCL_AMD_CFG_IPC_LIGHT_FENCE: *value = c.ipcLightFence; break;
        case HCCL_AMD_CFG_IPC_NT: *value = c.ipcNt; break;
        case HCCL_AMD_CFG_IPC_THREADS: *value = c.ipcThreads; break;
        case HCCL_AMD_CFG_IPC_TILE_KIB: *value = static_cast<int64_t>(c.ipcTileBytes >> 10); break;
        case HCCL_AMD_CFG_IPC_TIMEOUT_MS: *value = static_cast<int64_t>(c.ipcTimeoutMs); break;
        case HCCL_AMD_CFG_IPC_STAGING_MIB: *value = static_cast<int64_t>(c.ipcStagingBytes >> 20); break;
        case HCCL_AMD_CFG_IPC_TRACE: *value = c.ipcTrace; break;
        case HCCL_AMD_CFG_IPC_L2_SCRUB: *value = c.ipcL2Scrub; break;
        case HCCL_AMD_CFG_FOLD_TIMING: *value = c.foldTiming; break;
        case HCCL_AMD_CFG_IPC_LL_BYTES: *value = static_cast<int64_t>(c.ipcLlBytes); break;
        default: return HCCL_E_PARA;
    }
    return HCCL_SUCCESS;
}

uint64_t IpcTimeoutTicks() { return IpcTimeoutMsFromEnv() * 100000; }

}  // namespace hccl_amd
