"""Property-based fuzzing of the schedule builders (hypothesis): any operation x family x rank count x count x
pipelining granule x HCCL_BUFFSIZE x root, including the sizes where the ring and RHD spread over several rings /
instances, must (1) build identically shaped programs on every rank, (2) keep every transport group race-free, (3) stay
inside its declared staging and (4) compute the exact result when replayed by the oracle on int64 data whose sums
cannot round (each rank contributes a distinct power of two per element). Host only."""
import os

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import hccl_amd as H
from oracle import oracle as O

AR, RS, RED, AG = 0, 1, 2, 3
FAMILIES = {AR: [0, 1, 2, 3, 4, 5, 6, 8], RS: [0, 1, 3, 5, 6, 8], RED: [0, 1, 2, 5], AG: [0, 1, 3]}


@st.composite
def cases(draw):
    op_type = draw(st.sampled_from([AR, RS, RED, AG]))
    algo = draw(st.sampled_from(FAMILIES[op_type]))
    n = draw(st.sampled_from([2, 3, 4, 5, 6, 8]))
    div = n if op_type in (RS, AG) else 1
    count = draw(st.one_of(st.integers(1, 5_000 // div), st.integers(200_000 // div, 900_000 // div)))
    piece = draw(st.sampled_from([0, 128, 4096, 65536, 1 << 20]))
    root = draw(st.integers(0, n - 1))
    ccl = draw(st.sampled_from([None, "1", "3"]))  # HCCL_BUFFSIZE (MB): several executor loops when small
    return op_type, algo, n, count, piece, root, ccl


def _race_free(arr, nops):
    groups = {}
    for o in arr[:nops]:
        if o.kind in (2, 3):
            buf = o.srcBuf[0] if o.kind == 2 else o.dstBuf
            off = o.srcOff[0] if o.kind == 2 else o.dstOff
            groups.setdefault(o.group, []).append((buf, off, off + o.count, o.kind == 3))
    for acc in groups.values():
        acc.sort()
        for i in range(len(acc)):
            for j in range(i + 1, len(acc)):
                a, b = acc[i], acc[j]
                if b[0] != a[0] or b[1] >= a[2]:
                    break
                assert not (a[3] or b[3]), (a, b)


@settings(max_examples=150, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(cases())
def test_schedules_are_exact_race_free_and_bounded(case):
    op_type, algo, n, count, piece, root, ccl = case
    old = os.environ.get("HCCL_BUFFSIZE")
    if ccl is None:
        os.environ.pop("HCCL_BUFFSIZE", None)
    else:
        os.environ["HCCL_BUFFSIZE"] = ccl
    try:
        _check(op_type, algo, n, count, piece, root)
    finally:
        if old is None:
            os.environ.pop("HCCL_BUFFSIZE", None)
        else:
            os.environ["HCCL_BUFFSIZE"] = old


def _check(op_type, algo, n, count, piece, root):
    progs, used, scratch = [], set(), 0
    for r in range(n):
        arr, nops, u, se = H.build_schedule(op_type, algo, n, r, count, H.HcclDataType.INT64, root, piece)
        progs.append((arr, nops))
        used.add(u)
        scratch = max(scratch, se)
        _race_free(arr, nops)
        for o in arr[:nops]:  # staging references stay inside the declared staging
            refs = ([(o.dstBuf, o.dstOff)] if o.kind != 2 else []) + [(o.srcBuf[j], o.srcOff[j]) for j in range(o.nsrc)]
            for b, off in refs:
                if b == 2:
                    assert off + o.count <= se, (op_type, algo, n, count, piece, r)
    assert len(used) == 1
    in_count = count * n if op_type == RS else count
    out_count = count * n if op_type == AG else count
    idx = np.arange(in_count, dtype=np.int64)
    xs = [idx * (1 << 20) + (1 << r) for r in range(n)]
    bufs = [[x.copy(), np.zeros(out_count, np.int64), np.zeros(max(scratch, 1), np.int64)] for x in xs]
    assert O.replay(n, O.INT64, O.SUM, progs, bufs) == 0
    full = (1 << n) - 1
    for r in range(n):
        out = bufs[r][1]
        if op_type == AG:
            j = np.arange(out_count, dtype=np.int64)
            want = (j % count) * (1 << 20) + (np.int64(1) << (j // count))
        elif op_type == RED and r != root:
            want = np.zeros(out_count, np.int64)
        else:
            g = np.arange(count, dtype=np.int64) + (r * count if op_type == RS else 0)
            want = n * g * (1 << 20) + full
        assert np.array_equal(out, want), (op_type, algo, n, count, piece, root, r)
