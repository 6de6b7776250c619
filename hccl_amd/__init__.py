"""hccl_amd — MI355X-native HCCL reduce path (HcclAllReduce / HcclReduceScatter / HcclReduce).

The product is libhccl_amd.so: HIP kernels for gfx950 plus a C++ runtime (schedules, executor, RCCL transport)
behind the reference's C ABI (include/hccl.h). This Python module is a thin ctypes mirror of that ABI for tests
and benchmarks; torch supplies device memory and streams only. Names, argument meaning and return codes are the
C ABI's; every call raises HcclError on a non-success code.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import torch

from ._lib import (  # noqa: F401
    Algo,
    AivVariant,
    Config,
    HcclAmdIrOp,
    HcclAmdUnitPlan,
    HcclDataType,
    HcclError,
    HcclReduceOp,
    HcclResult,
    HcclRootInfo,
    IrKind,
    OpType,
    HCCL_ROOT_INFO_BYTES,
    IR_MAX_SRC,
    LIB_PATH,
    SIGNATURES,
    check,
    lib,
)

TORCH_TO_HCCL = {
    torch.int8: HcclDataType.INT8,
    torch.int16: HcclDataType.INT16,
    torch.int32: HcclDataType.INT32,
    torch.int64: HcclDataType.INT64,
    torch.uint64: HcclDataType.UINT64,
    torch.float16: HcclDataType.FP16,
    torch.bfloat16: HcclDataType.BFP16,
    torch.float32: HcclDataType.FP32,
    torch.float64: HcclDataType.FP64,
    # movable but not reducible (the reduce entries answer HCCL_E_NOT_SUPPORT, as CheckDataType does)
    torch.uint8: HcclDataType.UINT8,
    torch.uint16: HcclDataType.UINT16,
    torch.uint32: HcclDataType.UINT32,
    torch.float8_e4m3fn: HcclDataType.FP8E4M3,
    torch.float8_e5m2: HcclDataType.FP8E5M2,
}


def hccl_dtype(t: torch.Tensor) -> HcclDataType:
    try:
        return TORCH_TO_HCCL[t.dtype]
    except KeyError:
        raise TypeError(f"no HcclDataType for {t.dtype}") from None


def _stream(stream: Optional[torch.cuda.Stream]) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


# ----------------------------------------------------------------------------------------- local reduce primitive


def local_reduce(dst: torch.Tensor, src: torch.Tensor, op: int = HcclReduceOp.SUM, stream=None) -> None:
    """dst = src (op) dst on the GPU (HcclAmdLocalReduce = HcommLocalReduceOnThread)."""
    assert dst.numel() == src.numel() and dst.dtype == src.dtype
    check("HcclAmdLocalReduce",
          lib.HcclAmdLocalReduce(_ptr(dst), _ptr(src), dst.numel(), hccl_dtype(dst), int(op), _stream(stream)))


def local_reduce2(out: torch.Tensor, src: torch.Tensor, dst: torch.Tensor, op: int = HcclReduceOp.SUM,
                  stream=None) -> None:
    """out = src (op) dst."""
    assert out.numel() == src.numel() == dst.numel()
    check("HcclAmdLocalReduce2",
          lib.HcclAmdLocalReduce2(_ptr(out), _ptr(src), _ptr(dst), out.numel(), hccl_dtype(out), int(op),
                                  _stream(stream)))


def local_reduce_n(out: torch.Tensor, srcs: Sequence[torch.Tensor], op: int = HcclReduceOp.SUM, stream=None) -> None:
    """acc = srcs[0]; acc = srcs[j] (op) acc; out = acc."""
    arr = (ctypes.c_void_p * len(srcs))(*[s.data_ptr() for s in srcs])
    check("HcclAmdLocalReduceN",
          lib.HcclAmdLocalReduceN(_ptr(out), arr, len(srcs), out.numel(), hccl_dtype(out), int(op), _stream(stream)))


def set_reduce_launch(blocks_per_cu: int = 0, unroll: int = 0, cache_policy: int = 0) -> None:
    """0 restores each default; see HcclAmdSetReduceLaunch in include/hccl_amd.h."""
    check("HcclAmdSetReduceLaunch", lib.HcclAmdSetReduceLaunch(blocks_per_cu, unroll, cache_policy))


def set_fold_mode(mode: int = 0) -> None:
    """Operand pipelining of the n-ary fold (0 default, 1 serial, 2 prefetch, 3 all operands first);
    see HcclAmdSetFoldMode in include/hccl_amd.h."""
    check("HcclAmdSetFoldMode", lib.HcclAmdSetFoldMode(mode))


# ----------------------------------------------------------------------------------------- schedules


def build_schedule(op_type: int, algo: int, n_ranks: int, rank: int, count: int, dtype: int, root: int = 0,
                   piece_bytes: int = 0):
    """Returns (ops: ctypes array of HcclAmdIrOp, algo_used, scratch_elems)."""
    nops = ctypes.c_uint64(0)
    used = ctypes.c_int32(-1)
    scratch = ctypes.c_uint64(0)
    check("HcclAmdBuildSchedule",
          lib.HcclAmdBuildSchedule(op_type, algo, n_ranks, rank, count, int(dtype), root, piece_bytes, None, 0,
                                   ctypes.byref(nops), ctypes.byref(used), ctypes.byref(scratch)))
    arr = (HcclAmdIrOp * max(1, nops.value))()
    check("HcclAmdBuildSchedule",
          lib.HcclAmdBuildSchedule(op_type, algo, n_ranks, rank, count, int(dtype), root, piece_bytes, arr,
                                   nops.value, ctypes.byref(nops), ctypes.byref(used), ctypes.byref(scratch)))
    return arr, nops.value, used.value, scratch.value


def build_schedule_v(n_ranks: int, rank: int, counts: Sequence[int], displs: Sequence[int], dtype: int,
                     piece_bytes: int = 0):
    """ReduceScatterV schedule (HcclAmdBuildScheduleV): returns (ops, n_ops, scratch_elems)."""
    c = (ctypes.c_uint64 * n_ranks)(*counts)
    d = (ctypes.c_uint64 * n_ranks)(*displs)
    nops = ctypes.c_uint64(0)
    scratch = ctypes.c_uint64(0)
    check("HcclAmdBuildScheduleV", lib.HcclAmdBuildScheduleV(n_ranks, rank, c, d, int(dtype), piece_bytes, None, 0,
                                                             ctypes.byref(nops), ctypes.byref(scratch)))
    arr = (HcclAmdIrOp * max(1, nops.value))()
    check("HcclAmdBuildScheduleV", lib.HcclAmdBuildScheduleV(n_ranks, rank, c, d, int(dtype), piece_bytes, arr,
                                                             nops.value, ctypes.byref(nops), ctypes.byref(scratch)))
    return arr, nops.value, scratch.value


def select_algo(op_type: int, n_ranks: int, nbytes: int, special: bool = False) -> int:
    """The algorithm HCCL_AMD_ALGO_AUTO picks (HcclAmdSelectAlgo)."""
    return lib.HcclAmdSelectAlgo(int(op_type), n_ranks, nbytes, 1 if special else 0)


def select_aiv_algo(op_type: int, n_ranks: int, count: int, dtype: int, op: int, core_limit: int = 0,
                    strict: bool = False, aiv_only: bool = False):
    """(HcclAmdAivVariant, groupSize) the AIV engine takes (HcclAmdSelectAivAlgo); core_limit 0 = the default."""
    g = ctypes.c_uint32(1)
    flags = (1 if strict else 0) | (2 if aiv_only else 0)
    v = lib.HcclAmdSelectAivAlgo(int(op_type), n_ranks, count, int(dtype), int(op), core_limit, flags,
                                 ctypes.byref(g))
    return AivVariant(v), g.value


def executor_plan(ops, nops: int, elem_size: int, bases=(1 << 40, 2 << 40, 3 << 40)):
    """HcclAmdExecutorPlan: the executor's units for an IR program (from build_schedule), as a list of dicts."""
    base = (ctypes.c_uint64 * 3)(*bases)
    n = ctypes.c_uint64(0)
    check("HcclAmdExecutorPlan", lib.HcclAmdExecutorPlan(ops, nops, elem_size, base, None, 0, ctypes.byref(n)))
    units = (HcclAmdUnitPlan * max(1, n.value))()
    check("HcclAmdExecutorPlan", lib.HcclAmdExecutorPlan(ops, nops, elem_size, base, units, n.value, ctypes.byref(n)))
    return [{"stream": u.stream, "comm": bool(u.isComm), "first": u.firstOp, "num": u.numOps, "wait": u.waitUnit}
            for u in units[:n.value]]


def rccl_p2p_channels() -> tuple:
    """(NCCL_NCHANNELS_PER_PEER, NCCL_MIN_P2P_NCHANNELS) this process's RCCL communicators were created with
    (HcclAmdRcclP2pChannels; zeros before the first one)."""
    per = ctypes.c_uint32(0)
    mn = ctypes.c_uint32(0)
    check("HcclAmdRcclP2pChannels", lib.HcclAmdRcclP2pChannels(ctypes.byref(per), ctypes.byref(mn)))
    return per.value, mn.value


def l2_maintain(stream=None) -> None:
    """HcclAmdL2Maintain: system-scope write-back + invalidate of every XCD's L2, then wait (diagnostics)."""
    check("HcclAmdL2Maintain", lib.HcclAmdL2Maintain(_stream(stream)))


def diag_read_by_xcc(ptr: int, expect: torch.Tensor, non_temporal: bool = False, stream=None):
    """HcclAmdDiagReadByXcc over expect.numel() 4-byte words at device address ptr: per XCC id, the mismatching and the
    zero words summed over that XCD's workgroups (every workgroup reads the whole range), as two lists of 8."""
    out = torch.zeros(768, dtype=torch.int32, device=expect.device)
    words = expect.numel() * expect.element_size() // 4
    check("HcclAmdDiagReadByXcc", lib.HcclAmdDiagReadByXcc(ptr, _ptr(expect), words, 1 if non_temporal else 0,
                                                           _ptr(out), _stream(stream)))
    torch.cuda.synchronize()
    o = out.view(256, 3).cpu().tolist()
    bad, zero = [0] * 8, [0] * 8
    for b, z, x in o:
        bad[x & 7] += b
        zero[x & 7] += z
    return bad, zero


def ring_table(n_ranks: int) -> List[List[int]]:
    """The directed rings of HCCL_AMD_ALGO_RING (HcclAmdRingTable), as rank lists."""
    r = lib.HcclAmdRingTable(n_ranks, None, 0)
    buf = (ctypes.c_uint32 * max(1, r * n_ranks))()
    lib.HcclAmdRingTable(n_ranks, buf, r)
    return [list(buf[k * n_ranks:(k + 1) * n_ranks]) for k in range(r)]


def rhd_table(n_ranks: int) -> List[List[int]]:
    """The RHD instances (HcclAmdRhdTable): per instance, the real rank of each virtual rank."""
    r = lib.HcclAmdRhdTable(n_ranks, None, 0)
    buf = (ctypes.c_uint32 * max(1, r * n_ranks))()
    lib.HcclAmdRhdTable(n_ranks, buf, r)
    return [list(buf[k * n_ranks:(k + 1) * n_ranks]) for k in range(r)]


# ----------------------------------------------------------------------------------------- communicators


class Comm:
    """An HcclComm handle (RCCL-backed, or one rank of a loopback world)."""

    def __init__(self, handle: int):
        self.handle = ctypes.c_void_p(handle)

    @property
    def rank(self) -> int:
        v = ctypes.c_uint32(0)
        check("HcclGetRankId", lib.HcclGetRankId(self.handle, ctypes.byref(v)))
        return v.value

    @property
    def size(self) -> int:
        v = ctypes.c_uint32(0)
        check("HcclGetRankSize", lib.HcclGetRankSize(self.handle, ctypes.byref(v)))
        return v.value

    def set_algo(self, algo: int) -> None:
        check("HcclAmdCommSetAlgo", lib.HcclAmdCommSetAlgo(self.handle, int(algo)))

    def set_piece_bytes(self, nbytes: int) -> None:
        check("HcclAmdCommSetPieceBytes", lib.HcclAmdCommSetPieceBytes(self.handle, nbytes))

    def set_ipc_blocks(self, blocks: int) -> None:
        check("HcclAmdCommSetIpcBlocks", lib.HcclAmdCommSetIpcBlocks(self.handle, blocks))

    @property
    def last_algo(self) -> int:
        return lib.HcclAmdCommLastAlgo(self.handle)

    def set_config(self, key: int, value: int) -> None:
        """HcclAmdCommSetConfig: one entry of the communicator's configuration (Config; read from the environment when
        the communicator was created)."""
        check("HcclAmdCommSetConfig", lib.HcclAmdCommSetConfig(self.handle, int(key), int(value)))

    def fold_timing(self) -> dict:
        """HcclAmdCommFoldTiming: the folds of the last executor program while Config.FOLD_TIMING is on."""
        f, b = ctypes.c_uint64(0), ctypes.c_uint64(0)
        fu, su = ctypes.c_double(0), ctypes.c_double(0)
        check("HcclAmdCommFoldTiming", lib.HcclAmdCommFoldTiming(self.handle, ctypes.byref(f), ctypes.byref(b),
                                                                 ctypes.byref(fu), ctypes.byref(su)))
        return {"folds": f.value, "fold_bytes": b.value, "fold_us": fu.value, "span_us": su.value}

    def reload_config(self) -> None:
        """HcclAmdCommReloadConfig: the whole configuration from the environment again (test harnesses)."""
        check("HcclAmdCommReloadConfig", lib.HcclAmdCommReloadConfig(self.handle))

    def get_config(self, key: int) -> int:
        v = ctypes.c_int64(0)
        check("HcclAmdCommGetConfig", lib.HcclAmdCommGetConfig(self.handle, int(key), ctypes.byref(v)))
        return v.value

    def execute(self, ops, nops: int, send: torch.Tensor, recv: torch.Tensor, op: int = HcclReduceOp.SUM,
                single_stream: bool = False, stream=None, dtype=None) -> None:
        """HcclAmdCommExecute: run one rank's IR program (ctypes array of HcclAmdIrOp) on this communicator."""
        dt = hccl_dtype(send) if dtype is None else int(dtype)
        check("HcclAmdCommExecute", lib.HcclAmdCommExecute(self.handle, ops, nops, _ptr(send), _ptr(recv), dt, int(op),
                                                           1 if single_stream else 0, _stream(stream)))

    def scratch(self) -> tuple:
        """(device address, bytes) of the communicator's executor staging (HcclAmdCommScratch; diagnostics)."""
        p = ctypes.c_void_p(0)
        b = ctypes.c_uint64(0)
        check("HcclAmdCommScratch", lib.HcclAmdCommScratch(self.handle, ctypes.byref(p), ctypes.byref(b)))
        return p.value or 0, b.value

    def device_bytes(self) -> int:
        """Device bytes the library holds for this communicator now (HcclAmdCommDeviceBytes)."""
        b = ctypes.c_uint64(0)
        check("HcclAmdCommDeviceBytes", lib.HcclAmdCommDeviceBytes(self.handle, ctypes.byref(b)))
        return b.value

    def compile_stats(self) -> tuple:
        """(hits, misses) of the communicator's compiled-collective cache (HcclAmdCommCompileStats)."""
        h, m = ctypes.c_uint64(0), ctypes.c_uint64(0)
        check("HcclAmdCommCompileStats", lib.HcclAmdCommCompileStats(self.handle, ctypes.byref(h), ctypes.byref(m)))
        return h.value, m.value

    def graph_stats(self) -> tuple:
        """(launches, captures) of the communicator's executor graphs (HcclAmdCommGraphStats)."""
        la, ca = ctypes.c_uint64(0), ctypes.c_uint64(0)
        check("HcclAmdCommGraphStats", lib.HcclAmdCommGraphStats(self.handle, ctypes.byref(la), ctypes.byref(ca)))
        return la.value, ca.value

    def reduce_scatter_v(self, send: torch.Tensor, counts: Sequence[int], displs: Sequence[int], recv: torch.Tensor,
                         op: int = HcclReduceOp.SUM, stream=None) -> None:
        """HcclReduceScatterV: rank q's block of `send` is counts[q] elements at displs[q]."""
        n = len(counts)
        c = (ctypes.c_uint64 * n)(*counts)
        d = (ctypes.c_uint64 * n)(*displs)
        check("HcclReduceScatterV", lib.HcclReduceScatterV(_ptr(send), c, d, _ptr(recv), recv.numel(),
                                                           hccl_dtype(recv), int(op), self.handle, _stream(stream)))

    def ipc_status(self) -> int:
        """Status word of the IPC path (bit 0: a cross-rank barrier timed out on the last IPC AllReduce)."""
        v = ctypes.c_uint32(0)
        check("HcclAmdCommIpcStatus", lib.HcclAmdCommIpcStatus(self.handle, ctypes.byref(v)))
        return v.value

    def ipc_ll_launches(self) -> int:
        """HcclAmdCommIpcLlLaunches: one-sided launches of this communicator that ran in the LL form so far."""
        v = ctypes.c_uint32(0)
        check("HcclAmdCommIpcLlLaunches", lib.HcclAmdCommIpcLlLaunches(self.handle, ctypes.byref(v)))
        return v.value

    def ipc_trace(self):
        """Phase stamps of the last one-sided launch (HCCL_AMD_IPC_TRACE=1 at the first IPC call): a uint64 array
        [16 ranks][512 blocks][8 slots] of 100 MHz ticks and the workgroups per rank of that launch."""
        import numpy as np

        n = 16 * 512 * 8
        buf = (ctypes.c_uint64 * n)()
        b = ctypes.c_uint32(0)
        check("HcclAmdCommIpcTrace", lib.HcclAmdCommIpcTrace(self.handle, buf, n, ctypes.byref(b)))
        return np.frombuffer(buf, dtype=np.uint64).reshape(16, 512, 8).copy(), b.value

    def async_error(self) -> int:
        """HcclGetCommAsyncError: HCCL_E_TIMEOUT after an IPC barrier timeout, an RCCL asynchronous error, or 0."""
        v = ctypes.c_int(0)
        check("HcclGetCommAsyncError", lib.HcclGetCommAsyncError(self.handle, ctypes.byref(v)))
        return v.value

    def all_reduce(self, send: torch.Tensor, recv: torch.Tensor, op: int = HcclReduceOp.SUM, stream=None) -> None:
        check("HcclAllReduce", lib.HcclAllReduce(_ptr(send), _ptr(recv), send.numel(), hccl_dtype(send), int(op),
                                                 self.handle, _stream(stream)))

    def reduce_scatter(self, send: torch.Tensor, recv: torch.Tensor, op: int = HcclReduceOp.SUM,
                       stream=None) -> None:
        check("HcclReduceScatter", lib.HcclReduceScatter(_ptr(send), _ptr(recv), recv.numel(), hccl_dtype(send),
                                                         int(op), self.handle, _stream(stream)))

    def reduce(self, send: torch.Tensor, recv: torch.Tensor, root: int, op: int = HcclReduceOp.SUM,
               stream=None) -> None:
        check("HcclReduce", lib.HcclReduce(_ptr(send), _ptr(recv), send.numel(), hccl_dtype(send), int(op), root,
                                           self.handle, _stream(stream)))

    def all_gather(self, send: torch.Tensor, recv: torch.Tensor, stream=None) -> None:
        check("HcclAllGather", lib.HcclAllGather(_ptr(send), _ptr(recv), send.numel(), hccl_dtype(send),
                                                 self.handle, _stream(stream)))

    def destroy(self) -> None:
        if self.handle:
            check("HcclCommDestroy", lib.HcclCommDestroy(self.handle))
            self.handle = ctypes.c_void_p(0)


def get_root_info() -> bytes:
    ri = HcclRootInfo()
    check("HcclGetRootInfo", lib.HcclGetRootInfo(ctypes.byref(ri)))
    return bytes(ctypes.string_at(ctypes.addressof(ri), HCCL_ROOT_INFO_BYTES))


def comm_init_root_info(n_ranks: int, root_info: bytes, rank: int) -> Comm:
    ri = HcclRootInfo()
    ctypes.memmove(ctypes.addressof(ri), root_info, HCCL_ROOT_INFO_BYTES)
    h = ctypes.c_void_p(0)
    check("HcclCommInitRootInfo", lib.HcclCommInitRootInfo(n_ranks, ctypes.byref(ri), rank, ctypes.byref(h)))
    return Comm(h.value)


def ipc_idle_staging() -> int:
    """Bytes of the one-sided path's idle uncached blocks kept for reuse (HcclAmdIpcIdleStaging; they are never freed
    while the process runs)."""
    b = ctypes.c_uint64(0)
    check("HcclAmdIpcIdleStaging", lib.HcclAmdIpcIdleStaging(0, ctypes.byref(b)))
    return b.value


def comm_init_selfloop(n_ranks: int, rank: int = 0) -> Comm:
    """A one-GPU stand-in for rank `rank` of an n_ranks world: its schedules run through a one-rank RCCL communicator
    with every peer mapped onto itself (HcclAmdCommInitSelfLoop; harnesses only: the data no longer means the
    collective)."""
    h = ctypes.c_void_p(0)
    check("HcclAmdCommInitSelfLoop", lib.HcclAmdCommInitSelfLoop(n_ranks, rank, ctypes.byref(h)))
    return Comm(h.value)


def loopback_world(n_ranks: int) -> List[Comm]:
    arr = (ctypes.c_void_p * n_ranks)()
    check("HcclAmdCommInitLoopback", lib.HcclAmdCommInitLoopback(n_ranks, arr))
    return [Comm(arr[i]) for i in range(n_ranks)]


# HcclAmdHostAllGatherFn (include/hccl_amd.h)
HOST_ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                     ctypes.c_void_p)


def comm_init_host_exchange(n_ranks: int, rank: int, all_gather) -> Comm:
    """IPC-only communicator bootstrapped by `all_gather(bytes) -> list of n_ranks bytes objects` (e.g. over a
    torch.distributed gloo group). Its AllReduce is the one-sided IPC path."""

    def _cb(_ctx, mine, nbytes, out):
        try:
            parts = all_gather(ctypes.string_at(mine, nbytes))
            if len(parts) != n_ranks or any(len(b) != nbytes for b in parts):
                return 1
            ctypes.memmove(out, b"".join(parts), nbytes * n_ranks)
            return 0
        except Exception:  # noqa: BLE001  (an exception cannot cross the C boundary; the library reports failure)
            return 1

    fn = HOST_ALLGATHER_FN(_cb)
    h = ctypes.c_void_p(0)
    check("HcclAmdCommInitHostExchange",
          lib.HcclAmdCommInitHostExchange(n_ranks, rank, ctypes.cast(fn, ctypes.c_void_p), None, ctypes.byref(h)))
    c = Comm(h.value)
    c._keepalive = fn  # the library calls it for the communicator's lifetime
    return c


def rank_table_info(path: str, rank: int):
    """(n_ranks, device_id of rank) of a rank table file, validated as HcclCommInitClusterInfo validates it."""
    n = ctypes.c_uint32(0)
    dev = ctypes.c_int32(-1)
    check("HcclAmdRankTableInfo", lib.HcclAmdRankTableInfo(path.encode(), rank, ctypes.byref(n), ctypes.byref(dev)))
    return n.value, dev.value


def comm_init_cluster_info(path: str, rank: int) -> Comm:
    h = ctypes.c_void_p(0)
    check("HcclCommInitClusterInfo", lib.HcclCommInitClusterInfo(path.encode(), rank, ctypes.byref(h)))
    return Comm(h.value)


def comm_init_all(devices) -> List[Comm]:
    arr_dev = (ctypes.c_int32 * len(devices))(*devices)
    arr = (ctypes.c_void_p * len(devices))()
    check("HcclCommInitAll", lib.HcclCommInitAll(len(devices), arr_dev, arr))
    return [Comm(arr[i]) for i in range(len(devices))]


def last_bootstrap():
    """(stage, id_digest) of this process' last HcclCommInitClusterInfo: stage 0 = failed before the unique-id exchange
    completed, 1 = id exchanged over TCP, 2 = RCCL communicator created; id_digest = FNV-1a 64 of the exchanged id."""
    d = ctypes.c_uint64(0)
    st = ctypes.c_int32(0)
    check("HcclAmdLastBootstrap", lib.HcclAmdLastBootstrap(ctypes.byref(d), ctypes.byref(st)))
    return st.value, d.value


def bootstrap_exchange_id(path: str, rank: int, ident: bytes = b"") -> bytes:
    """The rank-table TCP exchange alone (host only): rank 0 serves `ident` (128 bytes), the others receive it."""
    buf = ctypes.create_string_buffer(ident.ljust(128, b"\0")[:128], 128)
    check("HcclAmdBootstrapExchangeId", lib.HcclAmdBootstrapExchangeId(path.encode(), rank, buf))
    return buf.raw


def pending_destroys() -> int:
    """Communicators whose HcclCommDestroy waits for the graphs captured on them to be destroyed."""
    return int(lib.HcclAmdCommPendingDestroys())


HOST_PROFILE_CATEGORIES = ("execute", "group", "fold", "copy", "record", "wait", "plan", "entry", "ipc")


def host_profile(reset: bool = True) -> dict:
    """Executor host time by category while HCCL_AMD_HOST_PROFILE=1: {category: (ns, calls)}."""
    n = len(HOST_PROFILE_CATEGORIES)
    ns = (ctypes.c_uint64 * n)()
    calls = (ctypes.c_uint64 * n)()
    check("HcclAmdHostProfile", lib.HcclAmdHostProfile(ns, calls, n, 1 if reset else 0))
    return {k: (ns[i], calls[i]) for i, k in enumerate(HOST_PROFILE_CATEGORIES)}
