"""ctypes/numpy front end of the CPU oracle (oracle/hccl_oracle.c). TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and only as the
checker (or as the timed CPU baseline). The product (hccl_amd / libhccl_amd.so) never imports it.
See hccl_oracle.c for the reference file:line each function restates.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import List, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")

# HcclDataType / HcclReduceOp numbering (include/hccl_types.h); kept local so the oracle imports nothing from the
# product package.
INT8, INT16, INT32, FP16, FP32, INT64, UINT64, UINT8, UINT16, UINT32, FP64, BFP16 = 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11
SUM, PROD, MAX, MIN = 0, 1, 2, 3

REDUCE_DTYPES = [INT8, INT16, INT32, INT64, UINT64, FP16, FP32, FP64, BFP16]
OPS = [SUM, PROD, MAX, MIN]
# storage type of each dtype (fp16 / bf16 are kept as raw uint16 bits)
NP_STORAGE = {
    INT8: np.int8, INT16: np.int16, INT32: np.int32, INT64: np.int64, UINT64: np.uint64,
    FP16: np.uint16, BFP16: np.uint16, FP32: np.float32, FP64: np.float64,
}
DTYPE_NAMES = {INT8: "int8", INT16: "int16", INT32: "int32", INT64: "int64", UINT64: "uint64", FP16: "fp16",
               FP32: "fp32", FP64: "fp64", BFP16: "bf16"}
OP_NAMES = {SUM: "sum", PROD: "prod", MAX: "max", MIN: "min"}
FLOAT_DTYPES = {FP16, FP32, FP64, BFP16}


def _ensure_built() -> None:
    src = os.path.join(_HERE, "hccl_oracle.c")
    if not os.path.exists(LIB_PATH) or (os.path.exists(src) and os.path.getmtime(src) > os.path.getmtime(LIB_PATH)):
        subprocess.run(["make", "-C", _HERE], check=True, stdout=subprocess.DEVNULL)


_ensure_built()
_lib = ctypes.CDLL(LIB_PATH)
_vp = ctypes.c_void_p
_lib.orc_fp16_to_fp32.restype = ctypes.c_float
_lib.orc_fp16_to_fp32.argtypes = [ctypes.c_uint16]
_lib.orc_fp32_to_fp16.restype = ctypes.c_uint16
_lib.orc_fp32_to_fp16.argtypes = [ctypes.c_float]
_lib.orc_bf16_to_fp32.restype = ctypes.c_float
_lib.orc_bf16_to_fp32.argtypes = [ctypes.c_uint16]
_lib.orc_fp32_to_bf16.restype = ctypes.c_uint16
_lib.orc_fp32_to_bf16.argtypes = [ctypes.c_float]
for _name in ("orc_aicpu_reduce", "orc_local_reduce"):
    getattr(_lib, _name).restype = ctypes.c_int
    getattr(_lib, _name).argtypes = [ctypes.c_int, ctypes.c_int, _vp, _vp, ctypes.c_uint64]
_lib.orc_reduce_n.restype = ctypes.c_int
_lib.orc_reduce_n.argtypes = [ctypes.c_int, ctypes.c_int, _vp, ctypes.POINTER(_vp), ctypes.c_uint32, ctypes.c_uint64]
_lib.orc_replay.restype = ctypes.c_int
_lib.orc_replay.argtypes = [ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_vp),
                            ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(_vp)]


def fp16_to_fp32(bits: int) -> float:
    return _lib.orc_fp16_to_fp32(bits)


def fp32_to_fp16(value: float) -> int:
    return _lib.orc_fp32_to_fp16(value)


def bf16_to_fp32(bits: int) -> float:
    return _lib.orc_bf16_to_fp32(bits)


def fp32_to_bf16(value: float) -> int:
    return _lib.orc_fp32_to_bf16(value)


def _p(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def aicpu_reduce(dtype: int, op: int, dst: np.ndarray, src: np.ndarray) -> int:
    """AicpuReduce (alg_data_trans_wrapper.cc:1254-1311): dst = src (op) dst in place. Returns the HcclResult."""
    return _lib.orc_aicpu_reduce(dtype, op, _p(dst), _p(src), dst.size)


def local_reduce(dtype: int, op: int, dst: np.ndarray, src: np.ndarray) -> np.ndarray:
    """LocalReduce semantics for every reduce dtype: dst = src (op) dst in place; returns dst."""
    assert dst.size == src.size
    ret = _lib.orc_local_reduce(dtype, op, _p(dst), _p(src), dst.size)
    if ret != 0:
        raise RuntimeError(f"orc_local_reduce returned {ret}")
    return dst


def reduce_n(dtype: int, op: int, srcs: Sequence[np.ndarray]) -> np.ndarray:
    """acc = srcs[0]; acc = srcs[j] (op) acc; returns acc (a new array)."""
    out = np.empty_like(srcs[0])
    arr = (_vp * len(srcs))(*[_p(s) for s in srcs])
    ret = _lib.orc_reduce_n(dtype, op, _p(out), arr, len(srcs), out.size)
    if ret != 0:
        raise RuntimeError(f"orc_reduce_n returned {ret}")
    return out


def replay(n_ranks: int, dtype: int, op: int, progs: Sequence, bufs: Sequence[Sequence[np.ndarray]]) -> int:
    """Replay per-rank IR programs (sequence of (ctypes HcclAmdIrOp array, nops)) over host buffers
    bufs[r] = [input, output, scratch]. Returns 0, an HcclResult code, or -1 on deadlock."""
    prog_ptrs = (_vp * n_ranks)(*[ctypes.cast(p[0], _vp) for p in progs])
    nops = (ctypes.c_uint64 * n_ranks)(*[p[1] for p in progs])
    flat: List[int] = []
    for r in range(n_ranks):
        for b in range(3):
            flat.append(_p(bufs[r][b]))
    buf_ptrs = (_vp * (3 * n_ranks))(*flat)
    return _lib.orc_replay(n_ranks, dtype, op, prog_ptrs, nops, buf_ptrs)


def equal_bits(dtype: int, got: np.ndarray, want: np.ndarray) -> bool:
    """Bit equality, except that any NaN matches any NaN (NaN payloads are not canonical across CPU and GPU;
    SURVEY.md §7 'Denormals / NaN')."""
    g = np.ascontiguousarray(got)
    w = np.ascontiguousarray(want)
    if g.shape != w.shape:
        return False
    if dtype in (FP32, FP64):
        gn, wn = np.isnan(g), np.isnan(w)
        return bool(np.array_equal(gn, wn) and np.array_equal(g.view(_uint(g))[~gn], w.view(_uint(w))[~wn]))
    if dtype == FP16:
        gn = ((g & 0x7C00) == 0x7C00) & ((g & 0x03FF) != 0)
        wn = ((w & 0x7C00) == 0x7C00) & ((w & 0x03FF) != 0)
        return bool(np.array_equal(gn, wn) and np.array_equal(g[~gn], w[~wn]))
    if dtype == BFP16:
        gn = ((g & 0x7F80) == 0x7F80) & ((g & 0x007F) != 0)
        wn = ((w & 0x7F80) == 0x7F80) & ((w & 0x007F) != 0)
        return bool(np.array_equal(gn, wn) and np.array_equal(g[~gn], w[~wn]))
    return bool(np.array_equal(g, w))


def _uint(a: np.ndarray):
    return {4: np.uint32, 8: np.uint64, 2: np.uint16}[a.itemsize]


def random_operands(dtype: int, count: int, seed: int, edge: bool = True, small_ints: bool = False):
    """Seeded operands for parity tests, with the IEEE / integer edge cases the reference's converters and
    std::max/std::min semantics distinguish (±0 ties, NaN, ±Inf, subnormals, max finite, wrap-around)."""
    rng = np.random.default_rng(seed)
    st = NP_STORAGE[dtype]
    if dtype == FP32:
        a = rng.uniform(-1, 1, count).astype(np.float32)
    elif dtype == FP64:
        a = rng.uniform(-1, 1, count)
    elif dtype == FP16:
        a = _fast_fp16(rng, count)
    elif dtype == BFP16:
        f = rng.uniform(-1, 1, count).astype(np.float32)
        a = (f.view(np.uint32) >> 16).astype(np.uint16)
    else:
        info = np.iinfo(st)
        if small_ints:
            lo, hi = max(info.min, -(1 << 20)), min(info.max, 1 << 20)
        else:
            lo, hi = info.min, info.max
        a = rng.integers(lo, hi, count, dtype=st, endpoint=True)
    edges = edge_values(dtype)
    a = np.ascontiguousarray(a.astype(st, copy=False))
    if edge and count >= 2 * len(edges):
        pos = rng.choice(count, size=len(edges), replace=False)
        a[pos] = edges
    return a


def edge_values(dtype: int) -> np.ndarray:
    """The values whose handling differs between plausible implementations of the reference's element rule."""
    st = NP_STORAGE[dtype]
    if dtype == FP32:
        return np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45, 1.17e-38, 3.4e38, -3.4e38, 1.0],
                        dtype=np.float32)
    if dtype == FP64:
        return np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, -5e-324, 2.2e-308, 1.7e308, -1.7e308, 1.0])
    if dtype == FP16:  # ±0, ±Inf, qNaN, sNaN, ±min subnormal, max subnormal, min normal, ±max, 1, 65504/2
        return np.array([0x0000, 0x8000, 0x7C00, 0xFC00, 0x7E00, 0x7C01, 0x0001, 0x8001, 0x03FF, 0x0400, 0x7BFF,
                         0xFBFF, 0x3C00, 0x77FF], dtype=np.uint16)
    if dtype == BFP16:
        return np.array([0x0000, 0x8000, 0x7F80, 0xFF80, 0x7FC0, 0x0001, 0x8001, 0x007F, 0x0080, 0x7F7F, 0xFF7F,
                         0x3F80], dtype=np.uint16)
    info = np.iinfo(st)
    return np.array([0, 1, info.max, info.min, info.max - 1, info.min + 1], dtype=st)


def edge_cross(dtype: int):
    """(src, dst) covering every ordered pair of edge values: exercises ties, NaN operand order and wrap."""
    e = edge_values(dtype)
    src = np.repeat(e, len(e))
    dst = np.tile(e, len(e))
    return np.ascontiguousarray(src), np.ascontiguousarray(dst)


def _fast_fp16(rng, count: int) -> np.ndarray:
    # numpy's float16 cast is IEEE round-to-nearest-even, the same as orc_fp32_to_fp16 for finite normal values
    return rng.uniform(-1, 1, count).astype(np.float32).astype(np.float16).view(np.uint16)
