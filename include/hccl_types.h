/*
 * hccl_types.h — MI355X-native drop-in for the CANN/hcomm HCCL type header.
 *
 * The reference includes <hccl/hccl_types.h> from the external CANN SDK
 * (/root/reference/include/hccl.h:14). That file is not in the reference tree, so the
 * numeric values below are pinned from the reference's own tables:
 *   - HcclDataType order: DATATYPE_SIZE_TABLE (/root/reference/src/ops/op_common/inc/alg_param.h:43-61)
 *     and VALID_HCCL_DATA_TYPES (/root/reference/src/common/hccl_common.h:60-67; value 13 is a gap,
 *     255 is RESERVED).
 *   - HcclReduceOp = {SUM, PROD, MAX, MIN, RESERVED} (/root/reference/src/common/hccl_common.h:124-129),
 *     numbered 0..4 as in the public CANN header.
 *   - HcclResult codes as in the public CANN header (HCCL_SUCCESS = 0, HCCL_E_PARA = 1, HCCL_E_PTR = 2,
 *     HCCL_E_NOT_SUPPORT = 5, HCCL_E_INTERNAL = 4, ...). tests/test_abi.py pins every value.
 *
 * Plain C: no HIP or torch types appear in any signature. aclrtStream is a hipStream_t passed as void*.
 */
#ifndef HCCL_AMD_HCCL_TYPES_H_
#define HCCL_AMD_HCCL_TYPES_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    HCCL_SUCCESS = 0,
    HCCL_E_PARA = 1,
    HCCL_E_PTR = 2,
    HCCL_E_MEMORY = 3,
    HCCL_E_INTERNAL = 4,
    HCCL_E_NOT_SUPPORT = 5,
    HCCL_E_NOT_FOUND = 6,
    HCCL_E_UNAVAIL = 7,
    HCCL_E_SYSCALL = 8,
    HCCL_E_TIMEOUT = 9,
    HCCL_E_OPEN_FILE_FAILURE = 10,
    HCCL_E_TCP_CONNECT = 11,
    HCCL_E_ROCE_CONNECT = 12,
    HCCL_E_TCP_TRANSFER = 13,
    HCCL_E_ROCE_TRANSFER = 14,
    HCCL_E_RUNTIME = 15,
    HCCL_E_DRV = 16,
    HCCL_E_PROFILING = 17,
    HCCL_E_CCE = 18,
    HCCL_E_NETWORK = 19,
    HCCL_E_AGAIN = 20,
    HCCL_E_REMOTE = 21,
    HCCL_E_SUSPENDING = 22,
    HCCL_E_RESERVED
} HcclResult;

typedef enum {
    HCCL_DATA_TYPE_INT8 = 0,
    HCCL_DATA_TYPE_INT16 = 1,
    HCCL_DATA_TYPE_INT32 = 2,
    HCCL_DATA_TYPE_FP16 = 3,
    HCCL_DATA_TYPE_FP32 = 4,
    HCCL_DATA_TYPE_INT64 = 5,
    HCCL_DATA_TYPE_UINT64 = 6,
    HCCL_DATA_TYPE_UINT8 = 7,
    HCCL_DATA_TYPE_UINT16 = 8,
    HCCL_DATA_TYPE_UINT32 = 9,
    HCCL_DATA_TYPE_FP64 = 10,
    HCCL_DATA_TYPE_BFP16 = 11,
    HCCL_DATA_TYPE_INT128 = 12,
    HCCL_DATA_TYPE_HIF8 = 14,
    HCCL_DATA_TYPE_FP8E4M3 = 15,
    HCCL_DATA_TYPE_FP8E5M2 = 16,
    HCCL_DATA_TYPE_FP8E8M0 = 17,
    HCCL_DATA_TYPE_RESERVED = 255
} HcclDataType;

typedef enum {
    HCCL_REDUCE_SUM = 0,
    HCCL_REDUCE_PROD = 1,
    HCCL_REDUCE_MAX = 2,
    HCCL_REDUCE_MIN = 3,
    HCCL_REDUCE_RESERVED = 4
} HcclReduceOp;

/* Opaque communicator handle (one per rank/device), as in CANN. */
typedef void* HcclComm;

/* aclrtStream on this platform is a hipStream_t carried as an untyped pointer. */
typedef void* aclrtStream;

/* Root info blob exchanged out of band before HcclCommInitRootInfo (CANN size). */
#define HCCL_ROOT_INFO_BYTES 4108
typedef struct HcclRootInfoDef {
    char internal[HCCL_ROOT_INFO_BYTES];
} HcclRootInfo;

#ifdef __cplusplus
}
#endif
#endif /* HCCL_AMD_HCCL_TYPES_H_ */
