"""ctypes binding of libhccl_amd.so (the C ABI declared in include/hccl.h and include/hccl_amd.h).

The library is the product: there is no Python or CPU fallback. If the shared object is missing, importing
this module raises. torch is imported first so that the HIP runtime torch ships is the one the library binds
to (both carry the soname libamdhip64.so.7 / librccl.so.1).
"""
from __future__ import annotations

import ctypes
import enum
import os

import torch  # noqa: F401  (loads the process' HIP runtime before the library)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libhccl_amd.so")


class HcclResult(enum.IntEnum):
    HCCL_SUCCESS = 0
    HCCL_E_PARA = 1
    HCCL_E_PTR = 2
    HCCL_E_MEMORY = 3
    HCCL_E_INTERNAL = 4
    HCCL_E_NOT_SUPPORT = 5
    HCCL_E_NOT_FOUND = 6
    HCCL_E_UNAVAIL = 7
    HCCL_E_SYSCALL = 8
    HCCL_E_TIMEOUT = 9
    HCCL_E_OPEN_FILE_FAILURE = 10
    HCCL_E_TCP_CONNECT = 11
    HCCL_E_ROCE_CONNECT = 12
    HCCL_E_TCP_TRANSFER = 13
    HCCL_E_ROCE_TRANSFER = 14
    HCCL_E_RUNTIME = 15
    HCCL_E_DRV = 16
    HCCL_E_PROFILING = 17
    HCCL_E_CCE = 18
    HCCL_E_NETWORK = 19
    HCCL_E_AGAIN = 20
    HCCL_E_REMOTE = 21
    HCCL_E_SUSPENDING = 22


class HcclDataType(enum.IntEnum):
    INT8 = 0
    INT16 = 1
    INT32 = 2
    FP16 = 3
    FP32 = 4
    INT64 = 5
    UINT64 = 6
    UINT8 = 7
    UINT16 = 8
    UINT32 = 9
    FP64 = 10
    BFP16 = 11
    INT128 = 12
    HIF8 = 14
    FP8E4M3 = 15
    FP8E5M2 = 16
    FP8E8M0 = 17
    RESERVED = 255


class HcclReduceOp(enum.IntEnum):
    SUM = 0
    PROD = 1
    MAX = 2
    MIN = 3
    RESERVED = 4


class Algo(enum.IntEnum):
    AUTO = 0
    MESH_ONESHOT = 1
    MESH_TWOSHOT = 2
    RING = 3
    RHD = 4
    NHR = 5
    ORDER_PRESERVED = 6
    IPC_TWOSHOT = 7
    MESH_CHUNK = 8
    IPC = 9
    AIV = 10
    AIV_ONLY = 11
    IPC_RHD = 12


class Config(enum.IntEnum):
    """HcclAmdConfigKey (include/hccl_amd.h): a communicator's configuration, read from the environment at creation."""
    DETERMINISTIC_STRICT = 0
    EXPANSION_MODE_AIV = 1
    AIV_CORE_LIMIT = 2
    SINGLE_STREAM_BYTES = 3
    SMALL_IPC_BYTES = 4
    PLAN_CACHE = 5
    GRAPH_CACHE = 6
    IPC_LIGHT_FENCE = 7
    IPC_NT = 8
    IPC_THREADS = 9
    IPC_TILE_KIB = 10
    IPC_TIMEOUT_MS = 11
    IPC_STAGING_MIB = 12
    IPC_TRACE = 14
    IPC_L2_SCRUB = 15
    FOLD_TIMING = 16
    IPC_LL_BYTES = 17


class AivVariant(enum.IntEnum):
    NOT_MATCHED = 0
    AR_ONESHOT = 1
    AR_TWOSHOT_LARGE = 2
    AR_TWOSHOT_SMALL = 3
    RS_BIGDATA = 4
    RS_LOCAL_TREE = 5


class OpType(enum.IntEnum):
    ALLREDUCE = 0
    REDUCE_SCATTER = 1
    REDUCE = 2
    ALLGATHER = 3
    REDUCE_SCATTER_V = 4


class IrKind(enum.IntEnum):
    COPY = 0
    REDUCE = 1
    SEND = 2
    RECV = 3


IR_MAX_SRC = 16
HCCL_ROOT_INFO_BYTES = 4108


class HcclAmdIrOp(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int32),
        ("peer", ctypes.c_int32),
        ("nsrc", ctypes.c_int32),
        ("group", ctypes.c_int32),
        ("count", ctypes.c_uint64),
        ("dstBuf", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("dstOff", ctypes.c_uint64),
        ("srcBuf", ctypes.c_int32 * IR_MAX_SRC),
        ("srcOff", ctypes.c_uint64 * IR_MAX_SRC),
    ]


class HcclAmdUnitPlan(ctypes.Structure):
    _fields_ = [
        ("stream", ctypes.c_int32),
        ("isComm", ctypes.c_int32),
        ("firstOp", ctypes.c_uint64),
        ("numOps", ctypes.c_uint64),
        ("waitUnit", ctypes.c_int64),
    ]


class HcclRootInfo(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * HCCL_ROOT_INFO_BYTES)]


# Every symbol the headers declare, with its ctypes signature. tests/test_abi.py checks the header and this
# table agree and that the library exports each one.
_vp = ctypes.c_void_p
_u32 = ctypes.c_uint32
_u64 = ctypes.c_uint64
_i32 = ctypes.c_int32
_res = ctypes.c_int
SIGNATURES = {
    # include/hccl.h
    "HcclAllReduce": (_res, [_vp, _vp, _u64, _i32, _i32, _vp, _vp]),
    "HcclReduceScatter": (_res, [_vp, _vp, _u64, _i32, _i32, _vp, _vp]),
    "HcclReduce": (_res, [_vp, _vp, _u64, _i32, _i32, _u32, _vp, _vp]),
    "HcclReduceScatterV": (_res, [_vp, _vp, _vp, _vp, _u64, _i32, _i32, _vp, _vp]),
    "HcclAllGather": (_res, [_vp, _vp, _u64, _i32, _vp, _vp]),
    "HcclGetRootInfo": (_res, [ctypes.POINTER(HcclRootInfo)]),
    "HcclCommInitRootInfo": (_res, [_u32, ctypes.POINTER(HcclRootInfo), _u32, ctypes.POINTER(_vp)]),
    "HcclCommDestroy": (_res, [_vp]),
    "HcclGetRankSize": (_res, [_vp, ctypes.POINTER(_u32)]),
    "HcclGetRankId": (_res, [_vp, ctypes.POINTER(_u32)]),
    "HcclGetCommAsyncError": (_res, [_vp, ctypes.POINTER(ctypes.c_int)]),
    # include/hccl_amd.h
    "HcclAmdLocalReduce": (_res, [_vp, _vp, _u64, _i32, _i32, _vp]),
    "HcclAmdLocalReduce2": (_res, [_vp, _vp, _vp, _u64, _i32, _i32, _vp]),
    "HcclAmdLocalReduceN": (_res, [_vp, ctypes.POINTER(_vp), _u32, _u64, _i32, _i32, _vp]),
    "HcclAmdSetReduceLaunch": (_res, [_u32, _u32, _u32]),
    "HcclAmdSetFoldMode": (_res, [_u32]),
    "HcclAmdDataTypeSize": (_u32, [_i32]),
    "HcclAmdGetErrorString": (ctypes.c_char_p, [_i32]),
    "HcclAmdSelectAlgo": (_i32, [_i32, _u32, _u64, _i32]),
    "HcclAmdBuildScheduleV": (_res, [_u32, _u32, ctypes.POINTER(_u64), ctypes.POINTER(_u64), _i32, _u64,
                                     ctypes.POINTER(HcclAmdIrOp), _u64, ctypes.POINTER(_u64), ctypes.POINTER(_u64)]),
    "HcclAmdSelectAivAlgo": (_i32, [_i32, _u32, _u64, _i32, _i32, _u32, _i32, ctypes.POINTER(_u32)]),
    "HcclAmdRingTable": (_i32, [_u32, ctypes.POINTER(_u32), _u32]),
    "HcclAmdRhdTable": (_i32, [_u32, ctypes.POINTER(_u32), _u32]),
    "HcclAmdBuildSchedule": (
        _res,
        [_i32, _i32, _u32, _u32, _u64, _i32, _u32, _u64, ctypes.POINTER(HcclAmdIrOp), _u64,
         ctypes.POINTER(_u64), ctypes.POINTER(_i32), ctypes.POINTER(_u64)],
    ),
    "HcclAmdExecutorPlan": (_res, [ctypes.POINTER(HcclAmdIrOp), _u64, _u32, ctypes.POINTER(_u64),
                                   ctypes.POINTER(HcclAmdUnitPlan), _u64, ctypes.POINTER(_u64)]),
    "HcclAmdCommInitLoopback": (_res, [_u32, ctypes.POINTER(_vp)]),
    "HcclAmdCommSetAlgo": (_res, [_vp, _i32]),
    "HcclAmdCommSetPieceBytes": (_res, [_vp, _u64]),
    "HcclAmdCommSetIpcBlocks": (_res, [_vp, _u32]),
    "HcclAmdCommLastAlgo": (_i32, [_vp]),
    "HcclAmdCommSetConfig": (_res, [_vp, _i32, ctypes.c_int64]),
    "HcclAmdCommGetConfig": (_res, [_vp, _i32, ctypes.POINTER(ctypes.c_int64)]),
    "HcclAmdCommReloadConfig": (_res, [_vp]),
    "HcclAmdCommFoldTiming": (_res, [_vp, ctypes.POINTER(_u64), ctypes.POINTER(_u64), ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(ctypes.c_double)]),
    "HcclAmdCommCompileStats": (_res, [_vp, ctypes.POINTER(_u64), ctypes.POINTER(_u64)]),
    "HcclAmdCommGraphStats": (_res, [_vp, ctypes.POINTER(_u64), ctypes.POINTER(_u64)]),
    "HcclAmdCommExecute": (_res, [_vp, ctypes.POINTER(HcclAmdIrOp), _u64, _vp, _vp, _i32, _i32, _i32, _vp]),
    "HcclAmdCommIpcStatus": (_res, [_vp, ctypes.POINTER(_u32)]),
    "HcclAmdCommIpcLlLaunches": (_res, [_vp, ctypes.POINTER(_u32)]),
    "HcclAmdCommIpcTrace": (_res, [_vp, ctypes.POINTER(_u64), _u64, ctypes.POINTER(_u32)]),
    "HcclAmdIpcTimeoutMs": (_u64, []),
    "HcclAmdCommInitHostExchange": (_res, [_u32, _u32, _vp, _vp, ctypes.POINTER(_vp)]),
    "HcclAmdRankTableInfo": (_res, [ctypes.c_char_p, _u32, ctypes.POINTER(_u32), ctypes.POINTER(ctypes.c_int32)]),
    "HcclCommInitClusterInfo": (_res, [ctypes.c_char_p, _u32, ctypes.POINTER(_vp)]),
    "HcclCommInitAll": (_res, [_u32, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(_vp)]),
    "HcclAmdLastBootstrap": (_res, [ctypes.POINTER(_u64), ctypes.POINTER(ctypes.c_int32)]),
    "HcclAmdBootstrapExchangeId": (_res, [ctypes.c_char_p, _u32, _vp]),
    "HcclAmdCommPendingDestroys": (_u32, []),
    "HcclAmdCommScratch": (_res, [_vp, ctypes.POINTER(_vp), ctypes.POINTER(_u64)]),
    "HcclAmdCommDeviceBytes": (_res, [_vp, ctypes.POINTER(_u64)]),
    "HcclAmdIpcIdleStaging": (_res, [_i32, ctypes.POINTER(_u64)]),
    "HcclAmdCommInitSelfLoop": (_res, [_u32, _u32, ctypes.POINTER(_vp)]),
    "HcclAmdL2Maintain": (_res, [_vp]),
    "HcclAmdRcclP2pChannels": (_res, [ctypes.POINTER(_u32), ctypes.POINTER(_u32)]),
    "HcclAmdDiagReadByXcc": (_res, [_vp, _vp, _u64, _i32, _vp, _vp]),
    "HcclAmdHostProfile": (_res, [ctypes.POINTER(_u64), ctypes.POINTER(_u64), _u32, _i32]),
}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make -C hccl_amd` or __graft_entry__.build() "
            "(there is no fallback implementation)"
        )
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue  # reported by tests/test_abi.py
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


class HcclError(RuntimeError):
    def __init__(self, fn: str, code: int):
        try:
            name = HcclResult(code).name
        except ValueError:
            name = str(code)
        super().__init__(f"{fn} returned {name}")
        self.code = code


def check(fn: str, code: int) -> None:
    if code != 0:
        raise HcclError(fn, code)
