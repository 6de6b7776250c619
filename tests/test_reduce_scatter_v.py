"""HcclReduceScatterV's schedule (HcclAmdBuildScheduleV) replayed by the CPU oracle against the mesh template's order
(tests/sched_ref.py reduce_scatter_v_o1; ins_temp_reduce_scatter_v_mesh_1D.cc:107-146), with ragged, empty, gapped,
reordered and overlapping blocks; sends and receives pair up, groups are race-free, and the entry checks follow
CheckReduceScatterVInputParam. Host only."""
import ctypes

import numpy as np
import pytest

import hccl_amd as H
from oracle import oracle as O
from tests import sched_ref as R

LAYOUTS = {
    "contiguous": lambda n: ([1000 + 37 * q for q in range(n)], None),
    "ragged_with_empty": lambda n: ([0 if q == 1 else 4099 * (q + 1) % 7001 + 1 for q in range(n)], None),
    "gapped": lambda n: ([513] * n, [q * 600 + 5 for q in range(n)]),
    "reordered": lambda n: ([777 + q for q in range(n)], [(n - 1 - q) * 800 for q in range(n)]),
    "overlapping": lambda n: ([1500] * n, [q * 100 for q in range(n)]),
}


def layout(name, n):
    counts, displs = LAYOUTS[name](n)
    if displs is None:
        displs = list(np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(int))
    return counts, displs


def replay(n, counts, displs, dtype, op, xs, piece_bytes=0):
    progs, scratch = [], 0
    for r in range(n):
        arr, nops, se = H.build_schedule_v(n, r, counts, displs, dtype, piece_bytes)
        progs.append((arr, nops))
        scratch = max(scratch, se)
    st = O.NP_STORAGE[dtype]
    bufs = [[x.copy(), np.zeros(max(1, counts[r]), st), np.zeros(max(scratch, 1), st)] for r, x in enumerate(xs)]
    assert O.replay(n, dtype, op, progs, bufs) == 0
    return [b[1][:counts[r]] for r, b in enumerate(bufs)], progs


@pytest.mark.parametrize("name", sorted(LAYOUTS))
@pytest.mark.parametrize("n", [2, 3, 4, 8])
@pytest.mark.parametrize("dtype,op", [(O.FP32, O.SUM), (O.FP16, O.SUM), (O.BFP16, O.MAX), (O.INT8, O.PROD),
                                      (O.INT64, O.MIN)])
def test_reduce_scatter_v_matches_mesh_order(name, n, dtype, op):
    counts, displs = layout(name, n)
    in_count = max(d + c for c, d in zip(counts, displs))
    xs = [O.random_operands(dtype, in_count, seed=70 + r, edge=False) for r in range(n)]
    got, progs = replay(n, counts, displs, dtype, op, xs, piece_bytes=2048)
    want = R.reduce_scatter_v_o1(dtype, op, xs, counts, displs)
    for r in range(n):
        assert O.equal_bits(dtype, got[r], want[r]), (name, r)
    for a in range(n):  # every SEND has its RECV (same size, same order) on the peer
        for b in range(n):
            if a != b:
                sends = [o.count for o in progs[a][0][:progs[a][1]] if o.kind == 2 and o.peer == b]
                recvs = [o.count for o in progs[b][0][:progs[b][1]] if o.kind == 3 and o.peer == a]
                assert sends == recvs, (a, b)
    for arr, nops in progs:  # groups race-free (test_schedules.test_groups_are_race_free)
        groups = {}
        for o in arr[:nops]:
            if o.kind in (2, 3):
                buf = o.srcBuf[0] if o.kind == 2 else o.dstBuf
                off = o.srcOff[0] if o.kind == 2 else o.dstOff
                groups.setdefault(o.group, []).append((buf, off, off + o.count, o.kind == 3))
        for acc in groups.values():
            for i in range(len(acc)):
                for j in range(i + 1, len(acc)):
                    x, y = acc[i], acc[j]
                    assert not (x[0] == y[0] and (x[3] or y[3]) and x[1] < y[2] and y[1] < x[2])


def test_reduce_scatter_v_single_rank_copies_its_block():
    xs = [np.arange(100, dtype=np.float32)]
    got, _ = replay(1, [30], [50], O.FP32, O.SUM, xs)
    assert np.array_equal(got[0], xs[0][50:80])


def test_reduce_scatter_v_entry_checks():
    """CheckReduceScatterVInputParam order (reduce_scatter_v_op.cc:155-183): stream, comm, sendCounts, sendDispls, then
    recvBuf when recvCount > 0 (HCCL_E_PTR)."""
    c = (ctypes.c_uint64 * 2)(1, 1)
    d = (ctypes.c_uint64 * 2)(0, 1)
    x = ctypes.c_void_p(0x1000)
    f = H.lib.HcclReduceScatterV
    assert f(x, c, d, x, 1, O.FP32, O.SUM, x, None) == H.HcclResult.HCCL_E_PTR       # stream
    assert f(x, c, d, x, 1, O.FP32, O.SUM, None, x) == H.HcclResult.HCCL_E_PTR       # comm
    assert f(x, None, d, x, 1, O.FP32, O.SUM, x, x) == H.HcclResult.HCCL_E_PTR       # sendCounts
    assert f(x, c, None, x, 1, O.FP32, O.SUM, x, x) == H.HcclResult.HCCL_E_PTR       # sendDispls
    assert f(x, c, d, None, 1, O.FP32, O.SUM, x, x) == H.HcclResult.HCCL_E_PTR       # recvBuf with recvCount > 0
    fake = ctypes.create_string_buffer(64)  # readable memory whose magic is not a communicator's
    assert f(x, c, d, x, 1, O.FP32, O.SUM, ctypes.addressof(fake), x) == H.HcclResult.HCCL_E_PARA


def test_reduce_scatter_v_rejects_wrapping_blocks():
    """A block whose end does not fit in 64-bit byte offsets would wrap the schedule onto other memory: refused with
    HCCL_E_PARA before any schedule is built."""
    counts = (ctypes.c_uint64 * 2)(8, 8)
    for displs in ((0, (1 << 64) - 4), (0, (1 << 62))):
        d = (ctypes.c_uint64 * 2)(*displs)
        n_ops = ctypes.c_uint64(0)
        assert H.lib.HcclAmdBuildScheduleV(2, 0, counts, d, O.FP32, 0, None, 0, ctypes.byref(n_ops),
                                           None) == H.HcclResult.HCCL_E_PARA
