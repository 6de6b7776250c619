// api_local.cc — C ABI of the local reduce primitive and shared helpers (include/hccl_amd.h).
#include <cstring>

#include "internal.h"

namespace hccl_amd {

uint32_t DataTypeSize(HcclDataType dt)
{
    // DATATYPE_SIZE_TABLE, /root/reference/src/ops/op_common/inc/alg_param.h:43-61 (value 13 is a gap).
    switch (dt) {
        case HCCL_DATA_TYPE_INT8:
        case HCCL_DATA_TYPE_UINT8:
        case HCCL_DATA_TYPE_HIF8:
        case HCCL_DATA_TYPE_FP8E4M3:
        case HCCL_DATA_TYPE_FP8E5M2:
        case HCCL_DATA_TYPE_FP8E8M0: return 1;
        case HCCL_DATA_TYPE_INT16:
        case HCCL_DATA_TYPE_UINT16:
        case HCCL_DATA_TYPE_FP16:
        case HCCL_DATA_TYPE_BFP16: return 2;
        case HCCL_DATA_TYPE_INT32:
        case HCCL_DATA_TYPE_UINT32:
        case HCCL_DATA_TYPE_FP32: return 4;
        case HCCL_DATA_TYPE_INT64:
        case HCCL_DATA_TYPE_UINT64:
        case HCCL_DATA_TYPE_FP64: return 8;
        case HCCL_DATA_TYPE_INT128: return 16;
        default: return 0;
    }
}

bool IsReduceDataType(HcclDataType dt)
{
    switch (dt) {
        case HCCL_DATA_TYPE_INT8:
        case HCCL_DATA_TYPE_INT16:
        case HCCL_DATA_TYPE_INT32:
        case HCCL_DATA_TYPE_INT64:
        case HCCL_DATA_TYPE_UINT64:
        case HCCL_DATA_TYPE_FP16:
        case HCCL_DATA_TYPE_FP32:
        case HCCL_DATA_TYPE_FP64:
        case HCCL_DATA_TYPE_BFP16: return true;
        default: return false;
    }
}

bool ParseExecTimeoutSeconds(const char* env, double* seconds)
{
    // ParseExecTimeout / IsValidNumberFormat (src/common/alg_env_config.cc:43-110): digits, optionally one '.' with
    // digits on both sides and at most two after it; at most UINT32_MAX. Unset or empty: not set.
    if (env == nullptr || env[0] == '\0') return false;
    const size_t len = std::strlen(env);
    const char* dot = std::strchr(env, '.');
    for (size_t i = 0; i < len; ++i) {
        if (env + i == dot) continue;
        if (env[i] < '0' || env[i] > '9') return false;
    }
    if (dot != nullptr) {
        const size_t decimals = len - size_t(dot - env) - 1;
        if (dot == env || decimals == 0 || decimals > 2) return false;
    }
    // parsed by hand: strtod would follow the process's LC_NUMERIC, where the decimal mark may be a comma
    uint64_t whole = 0;
    for (const char* q = env; *q != '\0' && q != dot; ++q) {
        whole = whole * 10 + uint64_t(*q - '0');
        if (whole > 4294967295ull) return false;
    }
    double frac = 0.0;
    if (dot != nullptr) {
        double scale = 0.1;
        for (const char* q = dot + 1; *q != '\0'; ++q, scale /= 10) frac += scale * (*q - '0');
    }
    const double v = double(whole) + frac;
    if (v > 4294967295.0) return false;
    *seconds = v;
    return true;
}

bool DebugEnabled()
{
    static int v = [] {
        const char* e = std::getenv("HCCL_AMD_DEBUG");
        return (e != nullptr && e[0] != '\0' && e[0] != '0') ? 1 : 0;
    }();
    return v != 0;
}

}  // namespace hccl_amd

using namespace hccl_amd;

extern "C" {

HcclResult HcclAmdLocalReduce(void* dst, const void* src, uint64_t count, HcclDataType dataType, HcclReduceOp op,
                              aclrtStream stream)
{
    // LocalReduce (alg_data_trans_wrapper.cc:901-928): size 0 is a success; otherwise dst = src (op) dst.
    if (count == 0) return HCCL_SUCCESS;
    if (dst == nullptr || src == nullptr) return HCCL_E_PTR;
    if (!IsReduceDataType(dataType)) return HCCL_E_NOT_SUPPORT;
    return LaunchReduce2(dst, src, dst, count, dataType, op, static_cast<hipStream_t>(stream));
}

HcclResult HcclAmdLocalReduce2(void* out, const void* src, const void* dst, uint64_t count, HcclDataType dataType,
                               HcclReduceOp op, aclrtStream stream)
{
    if (count == 0) return HCCL_SUCCESS;
    if (out == nullptr || src == nullptr || dst == nullptr) return HCCL_E_PTR;
    if (!IsReduceDataType(dataType)) return HCCL_E_NOT_SUPPORT;
    return LaunchReduce2(out, src, dst, count, dataType, op, static_cast<hipStream_t>(stream));
}

HcclResult HcclAmdLocalReduceN(void* out, const void* const* srcs, uint32_t nsrc, uint64_t count,
                               HcclDataType dataType, HcclReduceOp op, aclrtStream stream)
{
    if (count == 0) return HCCL_SUCCESS;
    if (out == nullptr || srcs == nullptr) return HCCL_E_PTR;
    if (nsrc == 0 || nsrc > HCCL_AMD_IR_MAX_SRC) return HCCL_E_PARA;
    for (uint32_t j = 0; j < nsrc; ++j) {
        if (srcs[j] == nullptr) return HCCL_E_PTR;
    }
    if (!IsReduceDataType(dataType)) return HCCL_E_NOT_SUPPORT;
    return LaunchReduceN(out, srcs, nsrc, count, dataType, op, static_cast<hipStream_t>(stream));
}

HcclResult HcclAmdSetReduceLaunch(uint32_t blocksPerCu, uint32_t unroll, uint32_t cachePolicy)
{
    return SetReduceLaunch(blocksPerCu, unroll, cachePolicy);
}

HcclResult HcclAmdSetFoldMode(uint32_t mode) { return SetFoldMode(mode); }

uint32_t HcclAmdDataTypeSize(HcclDataType dataType) { return DataTypeSize(dataType); }

const char* HcclAmdGetErrorString(HcclResult code)
{
    switch (code) {
        case HCCL_SUCCESS: return "HCCL_SUCCESS";
        case HCCL_E_PARA: return "HCCL_E_PARA";
        case HCCL_E_PTR: return "HCCL_E_PTR";
        case HCCL_E_MEMORY: return "HCCL_E_MEMORY";
        case HCCL_E_INTERNAL: return "HCCL_E_INTERNAL";
        case HCCL_E_NOT_SUPPORT: return "HCCL_E_NOT_SUPPORT";
        case HCCL_E_NOT_FOUND: return "HCCL_E_NOT_FOUND";
        case HCCL_E_UNAVAIL: return "HCCL_E_UNAVAIL";
        case HCCL_E_SYSCALL: return "HCCL_E_SYSCALL";
        case HCCL_E_TIMEOUT: return "HCCL_E_TIMEOUT";
        case HCCL_E_RUNTIME: return "HCCL_E_RUNTIME";
        case HCCL_E_DRV: return "HCCL_E_DRV";
        case HCCL_E_NETWORK: return "HCCL_E_NETWORK";
        case HCCL_E_AGAIN: return "HCCL_E_AGAIN";
        case HCCL_E_REMOTE: return "HCCL_E_REMOTE";
        case HCCL_E_SUSPENDING: return "HCCL_E_SUSPENDING";
        default: return "HCCL_E_UNKNOWN";
    }
}

}  // extern "C"
