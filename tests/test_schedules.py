"""Schedule IR (libhccl_amd.so, host-only code) replayed by the CPU oracle — no GPU needed.

For every collective x algorithm x rank count the per-rank programs from HcclAmdBuildSchedule are replayed by
orc_replay (one "sim world", the reference ST's idea with real data: test/st/algorithm/testcase/*.cc) and the
outputs are compared bit-for-bit with closed-form association orders written independently (tests/sched_ref.py).
This pins, e.g., that the two-shot AllReduce reproduces the reference's O2 order and the one-shot its O1 order.
It also covers config C1 (2 ranks, 1 MiB fp32 AllReduce on the host).
"""
import time

import numpy as np
import pytest

import hccl_amd as H
from oracle import oracle as O
from tests import sched_ref as R

AR, RS, RED, AG = 0, 1, 2, 3


def programs(op_type, algo, n, count, dtype, root=0, piece_bytes=0):
    progs, used = [], set()
    scratch = 0
    for r in range(n):
        arr, nops, algo_used, se = H.build_schedule(op_type, algo, n, r, count, dtype, root, piece_bytes)
        progs.append((arr, nops))
        used.add(algo_used)
        scratch = max(scratch, se)
    assert len(used) == 1
    return progs, used.pop(), scratch


def run(op_type, algo, n, count, dtype, op, root=0, piece_bytes=0, inplace=False, seed=0):
    progs, used, scratch = programs(op_type, algo, n, count, dtype, root, piece_bytes)
    in_count = count * n if op_type == RS else count
    st = O.NP_STORAGE[dtype]
    xs = [O.random_operands(dtype, in_count, seed=seed * 100 + r, edge=False, small_ints=True) for r in range(n)]
    bufs = []
    outs = []
    for r in range(n):
        inp = xs[r].copy()
        out = inp if inplace else np.zeros(count * n if op_type == AG else count, st)
        outs.append(out)
        bufs.append([inp, out, np.zeros(max(scratch, 1), st)])
    ret = O.replay(n, dtype, op, progs, bufs)
    assert ret == 0, f"replay returned {ret}"
    if inplace:
        outs = [o[:count] for o in outs]
    return used, xs, outs


CASES = [
    (AR, 1), (AR, 2), (AR, 3), (AR, 4), (AR, 5), (AR, 6), (AR, 8),
    (RS, 1), (RS, 3), (RS, 5), (RS, 6), (RS, 8),
    (RED, 1), (RED, 2), (RED, 5),
    (AG, 1), (AG, 3),
]


@pytest.mark.parametrize("count", [1, 7, 1000, 65537])
@pytest.mark.parametrize("n", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("op_type,algo", CASES)
def test_schedule_fp32_sum_matches_reference_order(op_type, algo, n, count):
    dtype, op = O.FP32, O.SUM
    used, xs, outs = run(op_type, algo, n, count, dtype, op, root=n - 1, piece_bytes=4096, seed=n)
    want = R.expected(op_type, used, dtype, op, xs, count, root=n - 1)
    for r in range(n):
        if op_type == RED and r != n - 1:
            assert not outs[r].any(), "Reduce must not write a non-root recvBuf"
            continue
        assert O.equal_bits(dtype, outs[r], want[r]), (op_type, used, n, count, r)


@pytest.mark.parametrize("dtype", [O.INT8, O.INT32, O.INT64, O.UINT64, O.FP16, O.BFP16, O.FP64],
                         ids=lambda v: O.DTYPE_NAMES[v])
@pytest.mark.parametrize("op", O.OPS, ids=lambda v: O.OP_NAMES[v])
@pytest.mark.parametrize("op_type,algo", CASES)
def test_schedule_dtypes_ops(op_type, algo, dtype, op):
    n, count = 4, 3001
    used, xs, outs = run(op_type, algo, n, count, dtype, op, root=1, piece_bytes=1024, seed=7)
    want = R.expected(op_type, used, dtype, op, xs, count, root=1)
    for r in range(n):
        if want[r] is None:
            continue
        assert O.equal_bits(dtype, outs[r], want[r]), (op_type, used, r)


def test_nhr_matches_survey_closed_form_o5():
    """SURVEY.md Appendix A, O5 for n = 8: slice r = ((x_r+x_{r+1})+(x_{r+2}+x_{r+3}))+((x_{r+4}+x_{r+5})+(x_{r+6}
    +x_{r+7})), every merge receiver partial (dst) (op) sender partial (src)."""
    n, count = 8, 8 * 1001
    used, xs, outs = run(AR, 5, n, count, O.FP32, O.SUM, piece_bytes=1024, seed=21)
    assert used == R.ALGO_NHR
    se = count // n
    for r in range(n):
        sl = slice(r * se, (r + 1) * se)
        x = lambda k: xs[(r + k) % n][sl]  # noqa: E731
        pair = lambda a, b: R.apply(O.FP32, O.SUM, b, a)  # noqa: E731  (a = dst, b = src)
        want = pair(pair(pair(x(0), x(1)), pair(x(2), x(3))), pair(pair(x(4), x(5)), pair(x(6), x(7))))
        for q in range(n):
            assert O.equal_bits(O.FP32, outs[q][sl], want), (r, q)


def test_order_preserved_tree_matches_o4():
    """SURVEY.md Appendix A, O4 for n = 8: ((x0+x4)+(x2+x6))+((x1+x5)+(x3+x7)), the same bits on every rank."""
    n, rc = 8, 3001
    used, xs, outs = run(RS, 6, n, rc, O.FP32, O.SUM, piece_bytes=2048, seed=41)
    assert used == R.ALGO_TREE
    for me in range(n):
        x = [xs[q][me * rc:(me + 1) * rc] for q in range(n)]
        pair = lambda a, b: R.apply(O.FP32, O.SUM, b, a)  # noqa: E731  (a = dst, b = src)
        want = pair(pair(pair(x[0], x[4]), pair(x[2], x[6])), pair(pair(x[1], x[5]), pair(x[3], x[7])))
        assert O.equal_bits(O.FP32, outs[me], want), me


@pytest.mark.parametrize("algo", [1, 2, 3, 4, 5, 6, 8])
def test_allreduce_inplace(algo):
    n, count = 4, 50000
    used, xs, outs = run(AR, algo, n, count, O.FP32, O.SUM, piece_bytes=8192, inplace=True, seed=3)
    want = R.expected(AR, used, O.FP32, O.SUM, xs, count)
    for r in range(n):
        assert O.equal_bits(O.FP32, outs[r], want[r])


def test_auto_selection_follows_reference_thresholds():
    """all_reduce_auto_selector.cc:545-550, reduce_scatter_auto_selector.cc:491, reduce_auto_selector.cc:319-324."""
    mib = 1 << 20
    assert programs(AR, 0, 8, 8 * mib // 4, O.FP32)[1] == R.ALGO_ONESHOT        # <= 8 MiB
    assert programs(AR, 0, 8, 8 * mib // 4 + 1, O.FP32)[1] == R.ALGO_TWOSHOT    # > 8 MiB
    assert programs(RS, 0, 8, 1024, O.FP32)[1] == R.ALGO_ONESHOT
    assert programs(RED, 0, 8, 8 * mib // 4 - 1, O.FP32)[1] == R.ALGO_ONESHOT   # < 8 MiB
    assert programs(RED, 0, 8, 8 * mib // 4, O.FP32)[1] == R.ALGO_TWOSHOT


def test_auto_selection_meshchunk_thresholds():
    """MeshChunk (all_reduce_auto_selector.cc:546-548: bytes * 8/n/n > 32 MiB, DEFAULT_RANK_SIZE = 8.0 in double;
    reduce_scatter_auto_selector.cc:491-495,512: recv bytes * (8/n)^2 > 16 MiB), never for 64-bit data (or PROD)."""
    mib = 1 << 20
    assert H.select_algo(AR, 8, 256 * mib, False) == R.ALGO_TWOSHOT              # 256 MiB * 1/8 = 32 MiB, not >
    assert H.select_algo(AR, 8, 256 * mib + 4, False) == R.ALGO_MESHCHUNK
    assert H.select_algo(AR, 8, 4 << 30, False) == R.ALGO_MESHCHUNK               # C3
    assert H.select_algo(AR, 8, 4 << 30, True) == R.ALGO_TWOSHOT                  # FP64 / INT64 / PROD
    assert H.select_algo(AR, 2, 16 * mib + 4, False) == R.ALGO_MESHCHUNK          # ratio 2 at n = 2
    assert H.select_algo(AR, 2, 16 * mib, False) == R.ALGO_TWOSHOT
    assert H.select_algo(AR, 3, 36 * mib, False) == R.ALGO_TWOSHOT                # 36 MiB * 8/9 = 32 MiB, not >
    assert H.select_algo(AR, 3, 37 * mib, False) == R.ALGO_MESHCHUNK
    assert H.select_algo(RS, 8, 16 * mib, False) == R.ALGO_ONESHOT
    assert H.select_algo(RS, 8, 16 * mib + 2, False) == R.ALGO_MESHCHUNK          # C4: 256 MiB per rank
    assert H.select_algo(RS, 4, 4 * mib + 2, False) == R.ALGO_MESHCHUNK          # ratio 4
    assert H.select_algo(RS, 8, 1 << 30, True) == R.ALGO_ONESHOT
    assert H.select_algo(RED, 8, 1 << 30, False) == R.ALGO_TWOSHOT
    # through the schedule builder (special = 64-bit data type)
    assert programs(AR, 0, 8, 64 * mib + 1, O.FP32)[1] == R.ALGO_MESHCHUNK
    assert programs(AR, 0, 8, 32 * mib + 1, O.FP64)[1] == R.ALGO_TWOSHOT


def test_meshchunk_o6_closed_form_n8():
    """O6 written out for n = 8: sub-slice j of owner t folds x_t, then x_{t+j+1}, ..., x_{t+7}, x_{t+1}, ..., x_{t+j}."""
    n, count = 8, 8 * 7 * 3 + 5
    used, xs, outs = run(AR, 8, n, count, O.FP32, O.SUM, piece_bytes=256, seed=61)
    assert used == R.ALGO_MESHCHUNK
    cs = -(-count // n)
    for t in range(n):
        b, e = t * cs, min(count, (t + 1) * cs)
        subs = R.even_subslices(e - b, n - 1)
        for j, (sb, se) in enumerate(subs):
            order = [t] + [(t + o) % n for o in list(range(j + 1, n)) + list(range(1, j + 1))]
            assert order == [t] + R.o6_peers(n, t, j)
            want = R.fold(O.FP32, O.SUM, [xs[q][b + sb:b + se] for q in order])
            for r in range(n):
                assert O.equal_bits(O.FP32, outs[r][b + sb:b + se], want), (t, j, r)


@pytest.mark.parametrize("op_type,n,count", [(AR, 3, 300007), (AR, 8, 140001), (RS, 3, 200003), (RS, 8, 70001),
                                              (AR, 2, 262147), (RS, 2, 300001)])
def test_meshchunk_follows_executor_loops(monkeypatch, op_type, n, count):
    """HCCL_BUFFSIZE = 1 MB: AllReduce loops of 512 KiB, ReduceScatter loops of 1 MiB / (n-1); every loop is sliced
    into chunks and sub-slices on its own, which decides each element's O6 rotation."""
    monkeypatch.setenv("HCCL_BUFFSIZE", "1")
    used, xs, outs = run(op_type, 8, n, count, O.FP32, O.SUM, piece_bytes=64 << 10, seed=n)
    want = R.expected(op_type, used, O.FP32, O.SUM, xs, count)
    for r in range(n):
        assert O.equal_bits(O.FP32, outs[r], want[r]), r


@pytest.mark.parametrize("n", list(range(1, 17)))
def test_ring_table_is_arc_disjoint_hamiltonian(n):
    """Every ring visits every rank once, no directed link (arc) carries two rings, and the count is the maximum
    (n-1: the complete digraph decomposes into Hamiltonian cycles for n != 4, 6 — Tillson) for n <= 8."""
    rings = H.ring_table(n)
    arcs = set()
    for c in rings:
        assert sorted(c) == list(range(n)), c
        if n > 1:
            for i in range(n):
                a = (c[i], c[(i + 1) % n])
                assert a not in arcs, (n, a)
                arcs.add(a)
    if n == 1:
        assert len(rings) == 1
    elif n <= 8:
        assert len(rings) == (n - 2 if n in (4, 6) else n - 1)
    else:
        import math
        assert len(rings) == sum(1 for k in range(1, n) if math.gcd(k, n) == 1)


@pytest.mark.parametrize("op_type,nbytes,links", [(AR, 64 << 20, 7), (AR, 1 << 20, 1), (AR, 3 << 20, 1),
                                                  (AR, 8 << 20, 2), (AR, 16 << 20, 3), (AR, 40 << 20, 5),
                                                  (RS, 64 << 20, 7), (RS, 1 << 20, 1), (AG, 64 << 20, 7),
                                                  (AG, 2 << 20, 1)])
def test_ring_count_grows_with_size(op_type, nbytes, links):
    """Rings spread over more links as the call grows (R^2 x 2n MiB <= 13.65 x bytes of the AllReduce buffer /
    ReduceScatter input / AllGather output), up to one ring per link at n = 8: then every rank sends to and receives
    from all 7 peers in every step."""
    assert R.ring_count(8, nbytes) == links
    count = nbytes // 4 if op_type == AR else nbytes // 4 // 8
    progs, used, _ = programs(op_type, 3, 8, count, O.FP32)
    assert used == R.ALGO_RING
    for arr, nops in progs:
        g = min(o.group for o in arr[:nops] if o.kind in (2, 3))
        first = [o for o in arr[:nops] if o.kind in (2, 3) and o.group == g]
        assert sorted(o.peer for o in first if o.kind == 2) == sorted(set(o.peer for o in first if o.kind == 2))
        assert len({o.peer for o in first if o.kind == 2}) == links
        assert len({o.peer for o in first if o.kind == 3}) == links


@pytest.mark.parametrize("n", [1, 2, 4, 8, 16])
def test_rhd_instances_cover_every_link_once_per_step(n):
    """Each RHD instance is a linear relabelling of the hypercube (virtual v -> real; XOR-compatible), and at every
    step the n-1 instances' partner vectors are all the nonzero vectors: every link carries exactly one instance."""
    t = H.rhd_table(n)
    assert len(t) == max(1, n - 1)
    m = n.bit_length() - 1
    for real in t:
        assert sorted(real) == list(range(n))
        for a in range(n):
            for b in range(n):
                assert real[a ^ b] == real[a] ^ real[b]  # linear over GF(2)
    for s in range(m):
        d = n >> (s + 1)
        vecs = sorted(real[d] for real in t)
        assert vecs == (list(range(1, n)) if n > 1 else [0])
    assert H.rhd_table(6) == [] and H.rhd_table(12) == []


@pytest.mark.parametrize("nbytes,links", [(1 << 10, 1), (1 << 20, 1), ((1 << 20) + 4, 1), (2 << 20, 2), (8 << 20, 4),
                                          (18 << 20, 6), ((49 << 20) // 2, 7), (4 << 30, 7)])
def test_rhd_instances_grow_with_size(nbytes, links):
    """RHD runs one instance for latency-bound calls and spreads over more links as the call grows (R^2 MiB <= 2 x
    bytes, at most n-1): the first group of every rank talks to exactly R peers."""
    assert R.rhd_instances(8, nbytes) == links
    progs, used, _ = programs(AR, 4, 8, nbytes // 4, O.FP32) if nbytes < (64 << 20) else (None, None, None)
    if progs is None:
        return
    assert used == R.ALGO_RHD
    for arr, nops in progs:
        g0 = [o for o in arr[:nops] if o.kind in (2, 3) and o.group == 0]
        assert len({o.peer for o in g0 if o.kind == 2}) == links and len({o.peer for o in g0 if o.kind == 3}) == links


def test_rhd_non_power_of_two_falls_back_to_ring():
    assert programs(AR, 4, 6, 1000, O.FP32)[1] == R.ALGO_RING


def test_schedule_scratch_is_bounded():
    """The staging a schedule addresses never exceeds the communicator's 2 x HCCL_BUFFSIZE (400 MiB default)."""
    for op_type, algo in CASES:
        for n in (2, 8):
            count = (4 << 30) // 4 // (n if op_type in (RS, AG) else 1)
            _, _, scratch = programs(op_type, algo, n, count, O.FP32)
            assert scratch * 4 <= 2 * (200 << 20), (op_type, algo, n, scratch)


# Orders that depend on which rank owns an element follow the reference's executor loops (a loop is at most
# min(transport bound, HCCL_BUFFSIZE / scratch multiple) bytes and is sliced on its own). With HCCL_BUFFSIZE = 1 MB:
# Reduce two-shot loops of 1 MiB / n, NHR AllReduce and Reduce loops of 1 MiB.
@pytest.mark.parametrize("op_type,algo,n,count", [
    (RED, 2, 3, 300001), (RED, 2, 8, 100003), (RED, 5, 5, 600001), (AR, 5, 6, 700001), (RS, 5, 3, 200003),
    (AR, 2, 4, 400003),
])
def test_ownership_orders_follow_executor_loops(monkeypatch, op_type, algo, n, count):
    monkeypatch.setenv("HCCL_BUFFSIZE", "1")
    used, xs, outs = run(op_type, algo, n, count, O.FP32, O.SUM, root=1, seed=11)
    assert used == algo
    want = R.expected(op_type, used, O.FP32, O.SUM, xs, count, root=1)
    for r in range(n):
        if op_type == RED and r != 1:
            continue
        assert O.equal_bits(O.FP32, outs[r], want[r]), r


def test_reduce_two_shot_slicing_is_balanced_not_aligned():
    """ReduceMesh1DTwoShot::CalcSlice gives the first count % n ranks one more element
    (reduce_mesh_1D_two_shot.cc:108-131); the 128-B aligned ceil split used by the AllReduce two-shot would make other
    ranks own (and fold first) some elements, which changes fp32 sums."""
    n, count = 3, 1000
    used, xs, outs = run(RED, 2, n, count, O.FP32, O.SUM, root=0, seed=3)
    want = R.reduce_twoshot(O.FP32, O.SUM, xs, 0)
    assert O.equal_bits(O.FP32, outs[0], want)
    aligned = np.empty_like(xs[0])
    for c, (b, e) in enumerate(R.chunk_bounds(count, n, 4)):
        if e > b:
            aligned[b:e] = R.fold(O.FP32, O.SUM, [xs[c][b:e]] + [xs[q][b:e] for q in range(n) if q != c])
    assert not O.equal_bits(O.FP32, outs[0], aligned)


def test_sends_and_recvs_pair_up():
    """Every SEND has the matching RECV (same size, same posting order) on the peer."""
    for op_type, algo in CASES:
        n = 5
        progs, _, _ = programs(op_type, algo, n, 4099, O.FP32, root=2, piece_bytes=2048)
        for a in range(n):
            for b in range(n):
                if a == b:
                    continue
                sends = [o.count for o in progs[a][0][:progs[a][1]] if o.kind == 2 and o.peer == b]
                recvs = [o.count for o in progs[b][0][:progs[b][1]] if o.kind == 3 and o.peer == a]
                assert sends == recvs, (op_type, algo, a, b)


@pytest.mark.parametrize("n", [2, 3, 5, 8])
@pytest.mark.parametrize("op_type,algo", CASES + [(AR, 7), (RS, 7)])
def test_every_output_holds_every_rank_once_at_its_offset(op_type, algo, n):
    """The reference ST's semantics check (test/st/algorithm/utils/src/hccl_verifier/.../allreduce_semantics_checker.cc:
    every output range is built from the INPUT of all rankSize ranks at the same offset), made numeric: rank r's
    element i is i * 2^20 + 2^r in int64, so the SUM at i is n * i * 2^20 + 2^n - 1 exactly when each rank
    contributes once and from offset i. A missing or repeated rank changes the low bits; a wrong offset the high ones.
    AllGather: block q of every output is rank q's input."""
    count, root = 10007, n // 2
    progs, used, scratch = programs(op_type, algo, n, count, O.INT64, root=root, piece_bytes=4096)
    in_count = count * n if op_type == RS else count
    idx = np.arange(in_count, dtype=np.int64)
    xs = [idx * (1 << 20) + (1 << r) for r in range(n)]
    bufs = [[x.copy(), np.zeros(count * n if op_type == AG else count, np.int64), np.zeros(max(scratch, 1), np.int64)]
            for x in xs]
    assert O.replay(n, O.INT64, O.SUM, progs, bufs) == 0
    full = (1 << n) - 1
    for r in range(n):
        out = bufs[r][1]
        if op_type == AG:
            assert np.array_equal(out, np.concatenate(xs)), r
        elif op_type == RS:
            g = np.arange(r * count, (r + 1) * count, dtype=np.int64)
            assert np.array_equal(out, n * g * (1 << 20) + full), r
        elif op_type == RED and r != root:
            assert not out.any()
        else:
            assert np.array_equal(out, n * np.arange(count, dtype=np.int64) * (1 << 20) + full), (r, used)


@pytest.mark.parametrize("inplace", [False, True])
def test_groups_are_race_free(inplace):
    """The reference ST's memory-conflict check (test/st/algorithm/utils/src/hccl_verifier/mem_conflict_check/)
    applied to the IR: the SEND/RECV records of one group run concurrently inside one RCCL group, so no two of
    them may touch overlapping bytes when either writes. (Ordering between groups and the reduce stream is derived
    by the executor from the same byte ranges, so it cannot race.) In-place aliases INPUT onto OUTPUT."""
    for op_type, algo in CASES:
        if inplace and op_type != AR:
            continue
        for n in (2, 3, 5, 8):
            count = 10007
            progs, _, _ = programs(op_type, algo, n, count, O.FP32, root=n - 1, piece_bytes=4096)
            for arr, nops in progs:
                groups = {}
                for o in arr[:nops]:
                    if o.kind in (2, 3):
                        buf = o.srcBuf[0] if o.kind == 2 else o.dstBuf
                        off = o.srcOff[0] if o.kind == 2 else o.dstOff
                        if inplace and buf == 0:
                            buf = 1
                        groups.setdefault(o.group, []).append((buf, off, off + o.count, o.kind == 3))
                for g, acc in groups.items():
                    for i in range(len(acc)):
                        for j in range(i + 1, len(acc)):
                            a, b = acc[i], acc[j]
                            if a[0] == b[0] and (a[3] or b[3]) and a[1] < b[2] and b[1] < a[2]:
                                raise AssertionError((op_type, algo, n, g, a, b))


def test_c1_sim_two_rank_1mib_allreduce():
    """Config C1: 2-rank AllReduce SUM, 1 MiB fp32, schedule replayed on the host (reference analogue:
    RunAllReduceCase, test/st/algorithm/testcase/all_reduce_testcase.cc:48-111, but with real data)."""
    count = (1 << 20) // 4
    t0 = time.perf_counter()
    used, xs, outs = run(AR, 0, 2, count, O.FP32, O.SUM, seed=11)
    dt = time.perf_counter() - t0
    assert used == R.ALGO_ONESHOT
    want = R.expected(AR, used, O.FP32, O.SUM, xs, count)
    for r in range(2):
        assert O.equal_bits(O.FP32, outs[r], want[r])
    assert dt < 30


@pytest.mark.parametrize("op_type,algo,n,nbytes", [
    (AR, 4, 8, (2 << 20) + 12),        # RHD, 2 instances
    (AR, 4, 8, (49 << 19) + 20),       # RHD, 7 instances
    (AR, 4, 4, (16 << 20) + 4),        # RHD, 3 instances at n = 4
    (AR, 3, 8, (8 << 20) + 28),        # ring, 2 rings
    (AR, 3, 8, (58 << 20) + 4),        # ring, 7 rings
    (AR, 3, 5, (40 << 20) + 12),       # ring, 4 rings at n = 5
    (RS, 3, 8, (58 << 20) + 8 * 12),   # ReduceScatter ring, 7 rings (input bytes)
])
def test_wide_rings_and_rhd_match_closed_form(op_type, algo, n, nbytes):
    """The ring and RHD at the sizes where they spread over several rings / instances (ragged counts, 1 MiB pieces):
    every output bit equals the closed form of sched_ref, which takes the same number of rings / instances."""
    count = nbytes // 4 if op_type == AR else nbytes // 4 // n
    used, xs, outs = run(op_type, algo, n, count, O.FP32, O.SUM, piece_bytes=1 << 20, seed=n + algo)
    assert used == algo
    want = R.expected(op_type, used, O.FP32, O.SUM, xs, count)
    for r in range(n):
        assert O.equal_bits(O.FP32, outs[r], want[r]), (op_type, algo, n, r)
