"""The executor's derived synchronisation is complete: for any schedule, any two units on different streams whose byte
ranges conflict (read-after-write, write-after-read, write-after-write) are ordered by the plan, through same-stream
program order and the cross-stream waits PlanUnits derives (it keeps only the latest conflicting unit per stream pair
and relies on transitivity; this checks that nothing is lost). Out-of-place and in-place (sendBuf == recvBuf) buffers,
property-based over operation x family x ranks x count x granule. Host only (HcclAmdExecutorPlan)."""
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import hccl_amd as H

AR, RS, RED, AG = 0, 1, 2, 3
FAMILIES = {AR: [1, 2, 3, 4, 5, 6, 8], RS: [1, 3, 5, 6, 8], RED: [1, 2, 5], AG: [1, 3]}
T = 1 << 40


def _ranges(arr, first, num, es, bases):
    out = []
    for i in range(first, first + num):
        o = arr[i]
        if o.kind == 2:
            out.append((bases[o.srcBuf[0]] + o.srcOff[0] * es, o.count * es, False))
        elif o.kind == 3:
            out.append((bases[o.dstBuf] + o.dstOff * es, o.count * es, True))
        else:
            out.append((bases[o.dstBuf] + o.dstOff * es, o.count * es, True))
            for j in range(o.nsrc):
                out.append((bases[o.srcBuf[j]] + o.srcOff[j] * es, o.count * es, False))
    return out


def _conflict(a, b):
    for (pa, la, wa) in a:
        for (pb, lb, wb) in b:
            if (wa or wb) and pa < pb + lb and pb < pa + la:
                return True
    return False


def _check(op_type, algo, n, rank, count, piece, inplace, drop_waits=False):
    es = 4
    arr, nops, _, _ = H.build_schedule(op_type, algo, n, rank, count, H.HcclDataType.FP32, 0, piece)
    bases = (T, T if inplace else 2 * T, 3 * T)
    units = H.executor_plan(arr, nops, es, bases)
    if drop_waits:
        for u in units:
            u["wait"] = -1
    rng = [_ranges(arr, u["first"], u["num"], es, bases) for u in units]
    before = []  # bit set of the units that happen before unit k
    last = {0: -1, 1: -1}
    for k, u in enumerate(units):
        hb = 0
        for p in (last[u["stream"]], u["wait"]):
            if p >= 0:
                hb |= before[p] | (1 << p)
        before.append(hb)
        last[u["stream"]] = k
    for b, ub in enumerate(units):
        for a in range(b):
            if units[a]["stream"] != ub["stream"] and not (before[b] >> a) & 1 and _conflict(rng[a], rng[b]):
                raise AssertionError((op_type, algo, n, rank, count, piece, inplace, a, b))


@st.composite
def cases(draw):
    op_type = draw(st.sampled_from([AR, RS, RED, AG]))
    algo = draw(st.sampled_from(FAMILIES[op_type]))
    n = draw(st.sampled_from([2, 3, 4, 8]))
    rank = draw(st.integers(0, n - 1))
    count = draw(st.integers(1, 400_000))
    piece = draw(st.sampled_from([0, 4096, 65536]))
    inplace = draw(st.booleans()) and op_type == AR
    return op_type, algo, n, rank, count, piece, inplace


@settings(max_examples=120, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(cases())
def test_every_cross_stream_hazard_is_ordered(case):
    _check(*case)


def test_c3_shapes_are_ordered():
    """The C3 shape's own plans (8 ranks, 4 GiB fp32) for the ring, MeshChunk and two-shot, in and out of place."""
    for algo in (3, 8, 2):
        for inplace in (False, True):
            _check(AR, algo, 8, 3, (4 << 30) // 4, 0, inplace)


def test_the_check_sees_a_missing_wait():
    """Negative control: the same plan without its cross-stream waits has unordered hazards."""
    import pytest
    with pytest.raises(AssertionError):
        _check(AR, 2, 8, 3, (64 << 20) // 4, 0, False, drop_waits=True)
