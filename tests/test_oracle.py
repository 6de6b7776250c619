"""Pins the CPU oracle (oracle/hccl_oracle.c) before anything is checked against it.

Sources of truth, in order:
  1. The reference's own numeric known answers: examples/02_collectives/{01_allreduce,04_reduce_scatter,05_reduce}/
     README_en.md "Sample Output" (8 ranks, x_r[i] = i, fp32 SUM) and the PyTorch sample
     examples/03_ai_framework/01_pytorch/hccl_pytorch_allreduce_test.py:30-38 (arange(world) -> world*arange).
  2. IEEE-754 binary16 conversion as implemented by numpy (exhaustive over all 65,536 fp16 patterns, and 2^20
     random fp32 patterns), which the reference converters (alg_data_trans_wrapper.cc:1077-1230) must agree with
     except where the reference deliberately differs (NaN payload handling; checked against the reference rule).
  3. numpy element-wise arithmetic with the reference's operand conventions (std::max/std::min(src, dst)).
  4. The reference's dtype routing (AicpuReduce :1254-1311 rejects INT16/BFP16 with HCCL_E_INTERNAL).
"""
import os

import numpy as np
import pytest

from oracle import oracle as O

HCCL_E_INTERNAL = 4


# ----------------------------------------------------------------------------------------------- reference KATs

def test_kat_allreduce_example_8_ranks():
    """examples/02_collectives/01_allreduce/README_en.md:59-70: every rank prints [0 8 16 24 32 40 48 56]."""
    xs = [np.arange(8, dtype=np.float32) for _ in range(8)]
    for order in (list(range(8)), [3, 0, 1, 2, 4, 5, 6, 7]):  # O2 and O1 (me = 3)
        got = O.reduce_n(O.FP32, O.SUM, [xs[r] for r in order])
        assert got.tolist() == [0, 8, 16, 24, 32, 40, 48, 56]


def test_kat_reduce_scatter_example():
    """examples/02_collectives/04_reduce_scatter/README_en.md: rank r prints [8 r] (recvCount = 1)."""
    xs = [np.arange(8, dtype=np.float32) for _ in range(8)]
    total = O.reduce_n(O.FP32, O.SUM, xs)
    for r in range(8):
        assert total[r] == 8 * r


def test_kat_reduce_example_root0():
    """examples/02_collectives/05_reduce/README_en.md: root 0 prints [0 8 ... 56]."""
    xs = [np.arange(8, dtype=np.float32) for _ in range(8)]
    assert O.reduce_n(O.FP32, O.SUM, xs).tolist() == [0, 8, 16, 24, 32, 40, 48, 56]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_kat_pytorch_sample(world):
    """hccl_pytorch_allreduce_test.py:30-38: arange(world) on every rank -> world * arange(world)."""
    xs = [np.arange(world, dtype=np.float32) for _ in range(world)]
    assert np.array_equal(O.reduce_n(O.FP32, O.SUM, xs), world * np.arange(world, dtype=np.float32))


# ----------------------------------------------------------------------------------------------- fp16 converters

def test_fp16_to_fp32_exhaustive():
    bits = np.arange(65536, dtype=np.uint32)
    got = np.array([O.fp16_to_fp32(int(b)) for b in bits], dtype=np.float32)
    want = bits.astype(np.uint16).view(np.float16).astype(np.float32)
    nan = np.isnan(want)
    assert np.array_equal(np.isnan(got), nan)
    assert np.array_equal(got[~nan].view(np.uint32), want[~nan].view(np.uint32))
    # the reference keeps NaN payloads: fp32 mantissa = fp16 mantissa << 13 (:1130-1138). Only quiet NaNs are
    # compared bit-wise: ctypes returns a C float through a double, which quiets signalling NaNs on x86.
    nb = bits[nan]
    quiet = (nb & 0x200) != 0
    nb = nb[quiet]
    got = got[nan][quiet]
    nan = slice(None)
    assert np.array_equal(got[nan].view(np.uint32), ((nb >> 15) << 31) | (0xFF << 23) | ((nb & 0x3FF) << 13))


def test_fp32_to_fp16_random_patterns():
    rng = np.random.default_rng(123)
    raw = rng.integers(0, 1 << 32, 1 << 20, dtype=np.uint64).astype(np.uint32)
    # bias towards the fp16 range so that rounding, subnormal and overflow paths are all hit
    near = (rng.integers(0x33000000, 0x47800000, 1 << 18, dtype=np.uint64).astype(np.uint32)
            | (rng.integers(0, 2, 1 << 18, dtype=np.uint64).astype(np.uint32) << 31))
    pats = np.concatenate([raw, near])
    f = pats.view(np.float32)
    got = np.array([O.fp32_to_fp16(float(x)) for x in f], dtype=np.uint16)
    with np.errstate(over="ignore"):
        want = f.astype(np.float16).view(np.uint16)
    nan = np.isnan(f)
    assert np.array_equal(got[~nan], want[~nan])
    # NaN rule (:1199-1207): sign | 0x7C00 | max(1, mantissa >> 13). Quiet NaNs only: the value reaches the C
    # function through a Python float (a double), which quiets signalling NaNs on x86.
    quiet = nan & ((pats & 0x400000) != 0)
    p = pats[quiet]
    m = (p & 0x7FFFFF) >> 13
    m[m == 0] = 1
    assert np.array_equal(got[quiet], (((p >> 31) << 15) | 0x7C00 | m).astype(np.uint16))


@pytest.mark.parametrize("value,bits", [
    (65504.0, 0x7BFF), (65519.99, 0x7BFF), (65520.0, 0x7C00), (2.0 ** -24, 0x0001), (2.0 ** -25, 0x0000),
    (2.0 ** -25 * 1.5, 0x0001), (3 * 2.0 ** -25, 0x0002), (2.0 ** -14 - 2.0 ** -25, 0x0400), (1e-40, 0x0000),
    (-0.0, 0x8000), (float("inf"), 0x7C00), (float("-inf"), 0xFC00),
])
def test_fp32_to_fp16_boundaries(value, bits):
    assert O.fp32_to_fp16(value) == bits


# ----------------------------------------------------------------------------------------------- element rule

def _np_rule(dtype, op, s, d):
    if dtype in (O.FP32, O.FP64):
        with np.errstate(all="ignore"):
            if op == O.SUM:
                return s + d
            if op == O.PROD:
                return s * d
            if op == O.MAX:
                return np.where(s < d, d, s)
            return np.where(d < s, d, s)
    if dtype in (O.INT8, O.INT16, O.INT32, O.INT64, O.UINT64):
        u = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[s.itemsize]
        with np.errstate(all="ignore"):
            if op == O.SUM:
                return (s.view(u) + d.view(u)).view(s.dtype)
            if op == O.PROD:
                return (s.view(u) * d.view(u)).view(s.dtype)
        if op == O.MAX:
            return np.where(s < d, d, s)
        return np.where(d < s, d, s)
    if dtype == O.FP16:
        fs, fd = s.view(np.float16).astype(np.float32), d.view(np.float16).astype(np.float32)
        with np.errstate(all="ignore"):
            if op == O.SUM:
                return (fs + fd).astype(np.float16).view(np.uint16)
            if op == O.PROD:
                return (fs * fd).astype(np.float16).view(np.uint16)
        if op == O.MAX:
            return np.where(fs < fd, d, s)
        return np.where(fd < fs, d, s)
    raise AssertionError


@pytest.mark.parametrize("op", O.OPS, ids=lambda v: O.OP_NAMES[v])
@pytest.mark.parametrize("dtype", [O.INT8, O.INT16, O.INT32, O.INT64, O.UINT64, O.FP16, O.FP32, O.FP64],
                         ids=lambda v: O.DTYPE_NAMES[v])
def test_element_rule_vs_numpy(dtype, op):
    for src, dst in (O.edge_cross(dtype),
                     (O.random_operands(dtype, 20011, seed=1), O.random_operands(dtype, 20011, seed=2))):
        want = _np_rule(dtype, op, src, dst)
        got = O.local_reduce(dtype, op, dst.copy(), src)
        assert O.equal_bits(dtype, got, want)


def test_max_min_tie_and_nan_return_src():
    """std::max(src, dst) / std::min(src, dst) return src on ties and whenever the comparison is false (NaN)."""
    s = np.array([0.0, -0.0, np.nan, 1.0], dtype=np.float32)
    d = np.array([-0.0, 0.0, 1.0, np.nan], dtype=np.float32)
    mx = O.local_reduce(O.FP32, O.MAX, d.copy(), s)
    mn = O.local_reduce(O.FP32, O.MIN, d.copy(), s)
    for got in (mx, mn):
        assert got[0] == 0 and not np.signbit(got[0])   # src = +0
        assert got[1] == 0 and np.signbit(got[1])       # src = -0
        assert np.isnan(got[2])                         # src = NaN
        assert got[3] == 1.0                            # src = 1 (NaN dst compares false)


def test_bf16_rule():
    """bf16 (parity unpinned: no in-tree reference arithmetic): fp32 compute, round-to-nearest-even."""
    src, dst = O.random_operands(O.BFP16, 30011, seed=3), O.random_operands(O.BFP16, 30011, seed=4)
    got = O.local_reduce(O.BFP16, O.SUM, dst.copy(), src)
    f = (src.astype(np.uint32) << 16).view(np.float32) + (dst.astype(np.uint32) << 16).view(np.float32)
    u = f.view(np.uint32)
    rne = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    nan = np.isnan(f)
    assert np.array_equal(got[~nan], rne[~nan])


def test_aicpu_reduce_routing():
    """AicpuReduce implements INT8/INT32/FP16/FP32/INT64/UINT64/FP64 only (:1264-1308)."""
    a = np.zeros(4, np.int16)
    assert O.aicpu_reduce(O.INT16, O.SUM, a, a.copy()) == HCCL_E_INTERNAL
    assert O.aicpu_reduce(O.BFP16, O.SUM, a.view(np.uint16), a.view(np.uint16).copy()) == HCCL_E_INTERNAL
    b = np.ones(4, np.int32)
    assert O.aicpu_reduce(O.INT32, O.PROD, b, b.copy()) == 0
    assert O.aicpu_reduce(O.INT32, 9, b, b.copy()) == HCCL_E_INTERNAL  # unknown op


def test_int_prod_wraps_like_reference():
    """int8 / int32 PROD go through unsigned wrap-around (:1329-1338)."""
    s = np.array([127, -128, 100], np.int8)
    d = np.array([127, -1, 3], np.int8)
    got = O.local_reduce(O.INT8, O.PROD, d.copy(), s)
    assert got.tolist() == [np.int8(np.uint8(127 * 127 % 256)), -128, np.int8(np.uint8(300 % 256))]


def test_reduce_n_is_an_ordered_fold():
    a = np.array([1e8], np.float32)
    b = np.array([1.0], np.float32)
    c = np.array([-1e8], np.float32)
    assert O.reduce_n(O.FP32, O.SUM, [a, b, c])[0] == np.float32(np.float32(1.0 + 1e8) + -1e8)
    assert O.reduce_n(O.FP32, O.SUM, [a, c, b])[0] == 1.0


def test_golden_file_matches_oracle():
    """The committed fixtures are exactly what the current oracle produces."""
    path = os.path.join(os.path.dirname(__file__), "golden", "local_reduce.npz")
    z = np.load(path, allow_pickle=False)
    for dtype in O.REDUCE_DTYPES:
        name = O.DTYPE_NAMES[dtype]
        src, dst = z[f"{name}_src"], z[f"{name}_dst"]
        for op in O.OPS:
            want = z[f"{name}_{O.OP_NAMES[op]}"]
            assert O.equal_bits(dtype, O.local_reduce(dtype, op, dst.copy(), src), want), (name, op)
