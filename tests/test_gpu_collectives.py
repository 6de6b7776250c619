"""GPU parity of HcclAllReduce / HcclReduceScatter / HcclReduce through the full executor.

n ranks live in one process on the one MI355X (HcclAmdCommInitLoopback): each rank has its own communicator, its
own streams and its own host thread, exactly as the reference's sample drives one thread per device
(examples/02_collectives/01_allreduce/main.cc:125-136); links are device-to-device copies, everything else —
schedules, stream/event dependencies, reduce kernels — is the code the RCCL path runs.

Every output is compared bit-for-bit with (a) the CPU oracle replaying the same schedule IR and (b) the closed-form
association order of the reference template (tests/sched_ref.py).
"""
import itertools
import os
import threading

import numpy as np
import pytest
import torch

import hccl_amd as H
from oracle import oracle as O
from tests import sched_ref as R
from tests._util import to_device, to_host

pytestmark = pytest.mark.gpu

AR, RS, RED, AG = 0, 1, 2, 3


@pytest.fixture(scope="module")
def worlds():
    cache = {}

    def get(n):
        # the worlds outlive a test, the environment a test sets (monkeypatch) does not: a communicator reads its
        # configuration when it is created, so every test's worlds read it again here
        if n not in cache:
            cache[n] = H.loopback_world(n)
        for c in cache[n]:
            c.reload_config()
        return cache[n]

    yield get
    torch.cuda.synchronize()
    for comms in cache.values():
        for c in comms:
            c.destroy()


def run_ranks(n, fn):
    errs = []

    def body(r):
        try:
            fn(r)
        except Exception as e:  # noqa: BLE001
            errs.append((r, e))

    th = [threading.Thread(target=body, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    assert not errs, errs


def collective(comms, op_type, algo, dtype, op, xs, count, root=0, piece_bytes=0, inplace=False, keep=None):
    """keep: a dict that receives the run's device buffers (keep["tensors"] = True keeps them alive, otherwise only
    their addresses are recorded and the blocks go back to torch's cache as usual)."""
    n = len(comms)
    sends = [to_device(dtype, x) for x in xs]
    zeros = np.zeros(count * n if op_type == AG else count, O.NP_STORAGE[dtype])
    recvs = [s if inplace else to_device(dtype, zeros) for s in sends]
    streams = [torch.cuda.Stream() for _ in range(n)]
    for c in comms:
        c.set_algo(algo)
        c.set_piece_bytes(piece_bytes)
    torch.cuda.synchronize()

    def body(r):
        if op_type == AR:
            comms[r].all_reduce(sends[r], recvs[r], op, streams[r])
        elif op_type == RS:
            comms[r].reduce_scatter(sends[r], recvs[r], op, streams[r])
        elif op_type == AG:
            comms[r].all_gather(sends[r], recvs[r], streams[r])
        else:
            comms[r].reduce(sends[r], recvs[r], root, op, streams[r])

    run_ranks(n, body)
    torch.cuda.synchronize()
    used = comms[0].last_algo
    outs = [to_host(dtype, r)[:count * n if op_type == AG else count] for r in recvs]
    if keep is not None:
        keep["send_ptrs"] = [hex(s.data_ptr()) for s in sends]
        keep["recv_ptrs"] = [hex(r.data_ptr()) for r in recvs]
        if keep.get("tensors"):
            keep["sends"], keep["recvs"] = sends, recvs
    for c in comms:
        c.set_algo(0)
        c.set_piece_bytes(0)
    return used, outs


def oracle_replay(op_type, algo, n, count, dtype, op, xs, root, piece_bytes):
    progs, scratch = [], 0
    for r in range(n):
        arr, nops, _, se = H.build_schedule(op_type, algo, n, r, count, dtype, root, piece_bytes)
        progs.append((arr, nops))
        scratch = max(scratch, se)
    st = O.NP_STORAGE[dtype]
    out_count = count * n if op_type == AG else count
    bufs = [[x.copy(), np.zeros(out_count, st), np.zeros(max(scratch, 1), st)] for x in xs]
    assert O.replay(n, dtype, op, progs, bufs) == 0
    return [b[1] for b in bufs]


CASES = [(AR, 1), (AR, 2), (AR, 3), (AR, 4), (AR, 5), (AR, 6), (AR, 7), (AR, 8), (RS, 1), (RS, 3), (RS, 5), (RS, 6),
         (RS, 7), (RS, 8), (RED, 1), (RED, 2), (RED, 5), (RED, 7), (AG, 1), (AG, 3)]


def ipc_status(comm):
    import ctypes
    v = ctypes.c_uint32(0)
    H.check("HcclAmdCommIpcStatus", H.lib.HcclAmdCommIpcStatus(comm.handle, ctypes.byref(v)))
    return v.value


@pytest.mark.parametrize("n", [2, 4, 8])
@pytest.mark.parametrize("count", [5, 4096, 1000003, 36 * (1 << 20) + 11])
def test_ipc_allreduce_o2_and_status(worlds, n, count):
    """The one-sided IPC AllReduce (one kernel, every rank's blocks in one launch on this GPU): bit-exact with the
    two-shot order O2, across several staging rounds (36 Mi fp32 > one 32 Mi-element round), barrier status clean."""
    comms = worlds(n)
    xs = [O.random_operands(O.FP32, count, seed=800 + r, edge=False) for r in range(n)]
    used, outs = collective(comms, AR, 7, O.FP32, O.SUM, xs, count)
    assert used == 7
    assert ipc_status(comms[0]) & 1 == 0
    want = R.expected(AR, R.ALGO_TWOSHOT, O.FP32, O.SUM, xs, count)
    for r in range(n):
        assert O.equal_bits(O.FP32, outs[r], want[r]), r


@pytest.mark.parametrize("n,count", [(2, (80 << 20) + 3), (4, (40 << 20) + 1), (8, 4099)])
def test_ipc_default_staging(monkeypatch, n, count):
    """The default large staging tier (HCCL_BUFFSIZE / 2 = 100 MiB areas since r06; 512 MiB before): two-shot IPC
    AllReduce bit-exact with order O2 over several staging rounds, barrier status clean."""
    monkeypatch.delenv("HCCL_AMD_IPC_STAGING_MIB", raising=False)
    comms = H.loopback_world(n)
    try:
        xs = [O.random_operands(O.FP32, count, seed=900 + r, edge=False) for r in range(n)]
        used, outs = collective(comms, AR, 7, O.FP32, O.SUM, xs, count)
        assert used == 7
        assert ipc_status(comms[0]) & 1 == 0
        want = R.expected(AR, R.ALGO_TWOSHOT, O.FP32, O.SUM, xs, count)
        for r in range(n):
            assert O.equal_bits(O.FP32, outs[r], want[r]), r
    finally:
        for c in comms:
            c.destroy()


@pytest.mark.parametrize("n,count", [(2, (3 << 20) + 5), (4, 1 << 20)])
def test_ipc_phase_trace(monkeypatch, n, count):
    """HCCL_AMD_IPC_TRACE=1 (r03): every block of every rank of the world's launch stamps its phases, in order
    (entry <= round <= phase 0 <= barrier 1 <= phase 1 <= barrier 2 <= phase 2 <= exit), and the output is still the
    two-shot's bits. Slots beyond the launch's blocks and ranks stay zero."""
    monkeypatch.setenv("HCCL_AMD_IPC_TRACE", "1")
    comms = H.loopback_world(n)
    try:
        for c in comms:
            c.set_ipc_blocks(32)
        xs = [O.random_operands(O.FP32, count, seed=950 + r, edge=False) for r in range(n)]
        used, outs = collective(comms, AR, 7, O.FP32, O.SUM, xs, count)
        assert used == 7
        want = R.expected(AR, R.ALGO_TWOSHOT, O.FP32, O.SUM, xs, count)
        for r in range(n):
            assert O.equal_bits(O.FP32, outs[r], want[r]), r
        st, blocks = comms[0].ipc_trace()
        assert blocks == 32
        a = st[:n, :blocks, :].astype(np.int64)
        assert (a > 0).all(), "a block or rank left a stamp unwritten"
        assert (np.diff(a, axis=2) >= 0).all(), "phase stamps out of order"
        assert not st[n:].any() and not st[:n, blocks:].any()
        # a world created without the variable has no trace
        monkeypatch.delenv("HCCL_AMD_IPC_TRACE")
        plain = H.loopback_world(2)
        try:
            collective(plain, AR, 7, O.FP32, O.SUM, xs[:2], count)
            with pytest.raises(H.HcclError):
                plain[0].ipc_trace()
        finally:
            for c in plain:
                c.destroy()
    finally:
        for c in comms:
            c.destroy()


@pytest.mark.parametrize("fence,threads", [("0", "256"), ("1", "512"), ("0", "512")])
@pytest.mark.parametrize("kind", [AR, RS, AG])
def test_ipc_barrier_variants(monkeypatch, fence, threads, kind):
    """The one-sided kernel with the system-scope barrier fences (HCCL_AMD_IPC_LIGHT_FENCE=0; the light fences, the
    waves' drains as the release and an agent-scope acquire, are the default the rest of the suite runs) and with
    512-thread workgroups (HCCL_AMD_IPC_THREADS): same bits as the schedule's order over several staging rounds and odd
    counts, barrier status clean."""
    monkeypatch.setenv("HCCL_AMD_IPC_LIGHT_FENCE", fence)
    monkeypatch.setenv("HCCL_AMD_IPC_THREADS", threads)
    monkeypatch.setenv("HCCL_AMD_IPC_STAGING_MIB", "16")
    n = 4
    comms = H.loopback_world(n)
    try:
        count = (5 << 20) + 3 if kind == AR else (3 << 20) + 7
        in_count = count * n if kind == RS else count
        xs = [O.random_operands(O.FP32, in_count, seed=970 + r, edge=False) for r in range(n)]
        used, outs = collective(comms, kind, 7, O.FP32, O.SUM, xs, count)
        assert used == 7
        assert ipc_status(comms[0]) & 1 == 0
        algo = R.ALGO_TWOSHOT if kind == AR else R.ALGO_IPC
        want = R.expected(kind, algo, O.FP32, O.SUM, xs, count)
        for r in range(n):
            assert O.equal_bits(O.FP32, outs[r], want[r]), r
    finally:
        for c in comms:
            c.destroy()


@pytest.mark.parametrize("op_type,n,count", [(RS, 2, (17 << 20) + 5), (RS, 4, 3), (RED, 4, (36 << 20) + 7),
                                              (RED, 3, 5)])
def test_ipc_reduce_scatter_and_reduce(worlds, op_type, n, count):
    """IPC ReduceScatter (order O1 per block owner) and Reduce (two-shot O1, chunk owner first, root gathers), with
    several pieces per chunk and with chunks smaller than one vector."""
    comms = worlds(n)
    root = n // 2
    in_count = count * n if op_type == RS else count
    xs = [O.random_operands(O.FP32, in_count, seed=600 + r, edge=False) for r in range(n)]
    used, outs = collective(comms, op_type, 7, O.FP32, O.SUM, xs, count, root=root)
    assert used == 7
    assert ipc_status(comms[0]) & 1 == 0
    want = R.expected(op_type, R.ALGO_IPC, O.FP32, O.SUM, xs, count, root=root)
    for r in range(n):
        if op_type == RED and r != root:
            assert not outs[r].any(), "non-root recvBuf written"
            continue
        assert O.equal_bits(O.FP32, outs[r], want[r]), r


@pytest.mark.parametrize("op_type,algo,n,count", [(RED, 2, 3, 300001), (RED, 5, 5, 600001), (AR, 5, 6, 700001),
                                                   (RED, 7, 4, 300001), (RED, 7, 3, 250003), (RS, 5, 3, 200003)])
def test_ownership_orders_follow_executor_loops(monkeypatch, op_type, algo, n, count):
    """With HCCL_BUFFSIZE = 1 MB the reference's executor loops are 1 MiB / n (Reduce two-shot, also on the IPC path)
    or 1 MiB (NHR): every loop is sliced on its own, which decides which rank's value is folded first."""
    monkeypatch.setenv("HCCL_BUFFSIZE", "1")
    comms = H.loopback_world(n)
    try:
        root = 1
        in_count = count * n if op_type == RS else count
        xs = [O.random_operands(O.FP32, in_count, seed=700 + r, edge=False) for r in range(n)]
        run = {"tensors": True}
        used, outs = collective(comms, op_type, algo, O.FP32, O.SUM, xs, count, root=root, keep=run)
        assert used == algo
        if algo == 7:
            assert ipc_status(comms[0]) & 1 == 0
        want = R.expected(op_type, used, O.FP32, O.SUM, xs, count, root=root)
        per_rank = [int(np.count_nonzero(outs[q].view(np.uint32) != want[q].view(np.uint32)))
                    if not (op_type == RED and q != root) else 0 for q in range(n)]
        diag = None
        if any(per_rank) and op_type != RED and algo != 7:
            from tests._stale_diag import _d2h, diagnose  # everything the failing run left behind, in the message
            diag = diagnose(comms, op_type, algo, xs, count, root, want, outs, run["sends"], run["recvs"])
            # the executor staging of each wrong rank as memory holds it now, at the first wrong elements and where the
            # program's receives landed (a later fold or copy would have read these words)
            diag["staging_now"] = {}
            for q in range(n):
                if not per_rank[q]:
                    continue
                bad = np.nonzero(outs[q].view(np.uint32) != want[q].view(np.uint32))[0]
                ptr, nbytes = comms[q].scratch()
                words = _d2h(ptr, nbytes).view(np.float32)
                arr, nops, _, _ = H.build_schedule(op_type, algo, n, q, count, O.FP32, root, 0)
                recv_offs = sorted({int(arr[i].dstOff) for i in range(nops)
                                    if arr[i].kind == H.IrKind.RECV and arr[i].dstBuf == 2})
                e = int(bad[0])
                starts = [int(bad[0])] + [int(bad[i]) for i in range(1, len(bad)) if bad[i] != bad[i - 1] + 1]
                runs = []
                for st in starts[:24]:
                    ln = 1
                    while st + ln in set(bad.tolist()):
                        ln += 1
                    # the operands whose float32 sum (rank order) is what the run's first element got
                    ops_ = [np.float32(x[q * count + st] if op_type == RS else x[st]) for x in xs]
                    fits = [list(c) for k in range(1, n + 1) for c in itertools.combinations(range(n), k)
                            if np.float32(sum(np.float32(ops_[i]) for i in c)) == outs[q][st]]
                    runs.append((st, ln, fits[:3]))
                diag.setdefault("bad_runs", {})[q] = runs
                # every run of zero words in the staging as memory holds it now (random operands are never 0): where
                # a receive's bytes were lost, and at what granularity (a 128-B line, a 4-KiB page, ...)
                zw = words.view(np.uint32) == 0
                edges = np.flatnonzero(np.diff(np.concatenate(([0], zw.astype(np.int8), [0]))))
                recs = [(int(arr[i].dstOff), int(arr[i].count)) for i in range(nops)
                        if arr[i].kind == H.IrKind.RECV and arr[i].dstBuf == 2]
                zero_runs = []
                for a0, a1 in zip(edges[0::2], edges[1::2]):
                    if a1 - a0 < 16:
                        continue
                    in_recv = [o for o, c in recs if o < a1 and a0 < o + c]
                    zero_runs.append({"off_B": int(a0) * 4, "len_B": int(a1 - a0) * 4, "addr_mod_4K": (ptr + int(a0) * 4) % 4096,
                                      "addr_mod_64K": (ptr + int(a0) * 4) % 65536, "in_recv_at": in_recv[:2]})
                diag["staging_now"][q] = {"at_bad": [float(words[int(b)]) for b in bad[:3]],
                                          "recv_offsets": recv_offs,
                                          "at_recv_plus_bad": {o: float(words[o + e]) for o in recv_offs
                                                               if o + e < len(words)},
                                          "operands_at_bad": [float(x[e]) for x in xs],
                                          "scratch": [hex(ptr), nbytes],
                                          "zero_runs": zero_runs[:40], "zero_runs_total": len(zero_runs)}
        for r in range(n):
            if op_type == RED and r != root:
                assert not outs[r].any(), "non-root recvBuf written"
                continue
            bad = np.nonzero(outs[r].view(np.uint32) != want[r].view(np.uint32))[0]
            assert not len(bad), (f"rank {r}: {len(bad)} bad, per rank {per_rank}, first {bad[:6].tolist()} last "
                                  f"{bad[-3:].tolist()}; got {outs[r][bad[:3]]!r} want {want[r][bad[:3]]!r}; "
                                  f"diagnosis {diag}")
    finally:
        torch.cuda.synchronize()
        for c in comms:
            c.destroy()


@pytest.mark.parametrize("op_type,n,count,buffsize", [
    (AR, 4, 4099, None),                    # one-shot O1
    (AR, 8, (9 << 20) // 4 + 3, None),      # two-shot O2 (8 MiB < bytes <= 256 MiB at n = 8)
    (AR, 2, (17 << 20) // 4 + 5, "4"),      # MeshChunk O6, loops of 2 MiB
    (AR, 3, (40 << 20) // 4 + 1, None),     # MeshChunk at n = 3: one loop, chunks not 16-B aligned
    (RS, 4, 1001, None),                    # mesh O1
    (RS, 4, (5 << 20) // 4 + 7, "4"),       # MeshChunk O6 with 4-KiB sub-slices, loops of 1 MiB
    (RS, 8, (3 << 20) // 4 + 3, None),      # MeshChunk at n = 8, one loop
    (RED, 4, 1003, None),                   # one-shot Reduce, root first
    (RED, 3, (9 << 20) // 4 + 1, None),     # two-shot Reduce
])
def test_ipc_follows_auto_family(monkeypatch, op_type, n, count, buffsize):
    """HCCL_AMD_ALGO_IPC runs the one-sided kernel in the order family the auto selector picks, so it gives the auto
    path's bits: compared with the closed form of that family and with the auto (RCCL-schedule) run itself."""
    if buffsize is not None:
        monkeypatch.setenv("HCCL_BUFFSIZE", buffsize)
    comms = H.loopback_world(n)
    try:
        root = n - 1
        in_count = count * n if op_type == RS else count
        xs = [O.random_operands(O.FP32, in_count, seed=520 + r, edge=False) for r in range(n)]
        family = H.select_algo(op_type, n, count * 4, False)
        ipc_run = {}
        if os.environ.get("HCCL_AMD_TEST_SKIP_IPC_RUN") == "1":  # diagnosis (tools/gpu_bisect_r04.sh): auto run only
            used, outs = 9, R.expected(op_type, family, O.FP32, O.SUM, xs, count, root=root)
        else:
            used, outs = collective(comms, op_type, 9, O.FP32, O.SUM, xs, count, root=root, keep=ipc_run)
        assert used == 9
        assert ipc_status(comms[0]) & 1 == 0
        auto_run = {"tensors": True}
        used_auto, outs_auto = collective(comms, op_type, 0, O.FP32, O.SUM, xs, count, root=root, keep=auto_run)
        assert used_auto == family
        want = R.expected(op_type, family, O.FP32, O.SUM, xs, count, root=root)
        diag = None
        if op_type != RED and any((outs_auto[r].view(np.uint32) != want[r].view(np.uint32)).any() for r in range(n)):
            from tests._stale_diag import diagnose
            diag = diagnose(comms, op_type, family, xs, count, root, want, outs_auto, auto_run["sends"],
                            auto_run["recvs"], history={"ipc_run": ipc_run, "auto_send_ptrs": auto_run["send_ptrs"],
                                                        "auto_recv_ptrs": auto_run["recv_ptrs"]})
        for r in range(n):
            if op_type == RED and r != root:
                assert not outs[r].any(), "non-root recvBuf written"
                continue
            bad = np.nonzero(outs[r].view(np.uint32) != want[r].view(np.uint32))[0]
            if len(bad):
                e = int(bad[0])
                per_rank = [int(np.count_nonzero(outs[q].view(np.uint32) != want[q].view(np.uint32))) for q in range(n)]
                prefix = np.cumsum(np.array([x[e] for x in xs], np.float64)).tolist()
                raise AssertionError(f"rank {r}: {len(bad)} bad, per rank {per_rank}, first {bad[:4].tolist()} "
                                     f"last {bad[-2:].tolist()}; at {e}: got {outs[r][e]!r} want {want[r][e]!r} "
                                     f"operands {[float(x[e]) for x in xs]} prefix sums {prefix}")
            diff = np.nonzero(outs_auto[r].view(np.uint32) != want[r].view(np.uint32))[0]
            assert not len(diff), (f"auto run, rank {r}: {len(diff)} elements differ from the closed form, first "
                                   f"{diff[:6].tolist()} last {diff[-3:].tolist()}; got {outs_auto[r][diff[:3]]!r} "
                                   f"want {want[r][diff[:3]]!r}; per rank "
                                   f"{[int(np.count_nonzero(outs_auto[q].view(np.uint32) != want[q].view(np.uint32))) for q in range(n)]}"
                                   f"; diagnosis {diag}")
    finally:
        torch.cuda.synchronize()
        for c in comms:
            c.destroy()


def _stale_line_bait(mib=9):
    """What preceded the observed failure: a world whose executor staging (cached, MTYPE RW) received raw operands,
    destroyed right away, so that its pages go back to the driver with lines still in the L2s. The next uncached IPC
    staging allocation may take those pages."""
    n, count = 4, (mib << 20) // 4 + 3
    comms = H.loopback_world(n)
    try:
        xs = [O.random_operands(O.FP32, count, seed=540 + r, edge=False) for r in range(n)]
        collective(comms, AR, 2, O.FP32, O.SUM, xs, count)
    finally:
        torch.cuda.synchronize()
        for c in comms:
            c.destroy()


def test_ipc_staging_survives_recycled_cached_pages():
    """Fresh uncached IPC staging right after a destroyed world released its cached staging. Context: r01's suite
    order made an 8-rank two-shot IPC AllReduce return a few stale operand lines in the owner's fold (fixed in r02: the
    barrier's dropped write-back wait). This test repeats the destroy-then-create pattern as a guard."""
    n, count = 8, (9 << 20) // 4 + 3
    xs = [O.random_operands(O.FP32, count, seed=530 + r, edge=False) for r in range(n)]
    want = R.expected(AR, R.ALGO_TWOSHOT, O.FP32, O.SUM, xs, count)
    for it in range(3):
        _stale_line_bait()
        comms = H.loopback_world(n)
        try:
            used, outs = collective(comms, AR, 7, O.FP32, O.SUM, xs, count)
            assert used == 7 and ipc_status(comms[0]) & 1 == 0
            for r in range(n):
                bad = np.nonzero(outs[r].view(np.uint32) != want[r].view(np.uint32))[0]
                assert len(bad) == 0, (it, r, len(bad), bad[:4].tolist())
        finally:
            torch.cuda.synchronize()
            for c in comms:
                c.destroy()


@pytest.mark.parametrize("dtype", [torch.uint8, torch.float16, torch.float32, torch.float64, torch.int64],
                         ids=str)
@pytest.mark.parametrize("n,count", [(2, 1), (3, 5), (4, 4099), (8, 100003), (2, (36 << 20) + 11)])
@pytest.mark.parametrize("inplace", [False, True])
def test_ipc_allgather(worlds, dtype, n, count, inplace):
    """AllGather on the IPC kernel (pure data movement: any dtype, including the non-reducible uint8): rank r's
    input lands in block r of every output (all_gather_op.cc semantics), across several staging rounds, in place
    (sendBuf = recvBuf + r * count) or not."""
    if count > (1 << 20) and dtype != torch.float32:
        pytest.skip("multi-round case runs once, in fp32")
    comms = worlds(n)
    g = torch.Generator(device="cuda").manual_seed(900 + n)
    full = torch.randint(0, 256, (n * count * dtype.itemsize,), device="cuda", dtype=torch.uint8,
                         generator=g).view(dtype)
    recvs = [torch.zeros(n * count, dtype=dtype, device="cuda") for _ in range(n)]
    sends = []
    for r in range(n):
        if inplace:
            recvs[r][r * count:(r + 1) * count] = full[r * count:(r + 1) * count]
            sends.append(recvs[r][r * count:(r + 1) * count])
        else:
            sends.append(full[r * count:(r + 1) * count].clone())
    streams = [torch.cuda.Stream() for _ in range(n)]
    for c in comms:
        c.set_algo(H.Algo.IPC)
    torch.cuda.synchronize()
    try:
        run_ranks(n, lambda r: comms[r].all_gather(sends[r], recvs[r], streams[r]))
        torch.cuda.synchronize()
        assert comms[0].last_algo == H.Algo.IPC
        assert ipc_status(comms[0]) & 1 == 0
        want = full.view(torch.uint8)
        for r in range(n):
            assert torch.equal(recvs[r].view(torch.uint8), want), r
    finally:
        for c in comms:
            c.set_algo(0)


@pytest.mark.parametrize("dtype,algo", [(O.INT8, 7), (O.INT8, 9), (O.FP16, int(H.Algo.IPC_RHD))])
def test_ipc_blocks_capped_at_resident(worlds, monkeypatch, dtype, algo):
    """Co-residency guard (ipc.cc RunIpcPlan, IpcResidentBlocks): the int8 IPC kernel uses 191 VGPRs, so the GPU holds
    2 of its workgroups per CU; an 8-rank loopback world asking for 256 blocks per rank (2,048) would wait forever
    for blocks that cannot start. The launch is capped at the resident count, and the result is exact."""
    monkeypatch.setenv("HCCL_AMD_IPC_TIMEOUT_MS", "20000")  # a stuck barrier fails the test, never hangs the box
    n, count = 8, (24 << 20) + 3
    comms = worlds(n)
    xs = [O.random_operands(dtype, count, seed=990 + r, edge=False, small_ints=True) for r in range(n)]
    for c in comms:
        c.set_ipc_blocks(256)
    try:
        used, outs = collective(comms, AR, algo, dtype, O.SUM, xs, count)
    finally:
        for c in comms:
            c.set_ipc_blocks(0)
    assert used == algo
    assert ipc_status(comms[0]) & 1 == 0
    if dtype == O.INT8:
        want = R.fold(dtype, O.SUM, xs)  # wrap-around integer sums: every order gives these bits
        for r in range(n):
            assert O.equal_bits(dtype, outs[r], want), r
    else:
        want = oracle_replay(AR, R.ALGO_RHD, n, count, dtype, O.SUM, xs, 0, 0)
        for r in range(n):
            assert O.equal_bits(dtype, outs[r], want[r]), r


@pytest.mark.parametrize("shift", [(1, 1), (0, 3), (2, 0)])
def test_ipc_unaligned_buffers(worlds, shift):
    """Buffers not 16-B aligned still run the IPC kernel (element-wise accesses to the user buffers; the path choice
    never depends on one rank's local buffers, so ranks cannot diverge) and give order O2."""
    n, count = 4, 10001
    si, so = shift
    comms = worlds(n)
    xs = [O.random_operands(O.FP32, count + si, seed=900 + r, edge=False) for r in range(n)]
    sends = [to_device(O.FP32, x)[si:] for x in xs]
    recvs = [torch.zeros(count + so, device="cuda")[so:] for _ in range(n)]
    streams = [torch.cuda.Stream() for _ in range(n)]
    for c in comms:
        c.set_algo(7)
    torch.cuda.synchronize()
    run_ranks(n, lambda r: comms[r].all_reduce(sends[r], recvs[r], O.SUM, streams[r]))
    torch.cuda.synchronize()
    assert comms[0].last_algo == R.ALGO_IPC
    assert ipc_status(comms[0]) & 1 == 0
    for c in comms:
        c.set_algo(0)
    want = R.expected(AR, R.ALGO_TWOSHOT, O.FP32, O.SUM, [x[si:].copy() for x in xs], count)
    for r in range(n):
        assert O.equal_bits(O.FP32, to_host(O.FP32, recvs[r]), want[r]), r


def test_hccl_deterministic_strict_selects_tree(worlds, monkeypatch):
    """HCCL_DETERMINISTIC=strict + fp32 SUM + more than 2 ranks selects the order-preserved tree (O4) for
    AllReduce and ReduceScatter (order_preserved_common.h:63-73); int32 or 2 ranks keep the default."""
    monkeypatch.setenv("HCCL_DETERMINISTIC", "strict")
    n, count = 4, 70001
    comms = worlds(n)
    xs = [O.random_operands(O.FP32, count, seed=600 + r, edge=False) for r in range(n)]
    used, outs = collective(comms, AR, 0, O.FP32, O.SUM, xs, count)
    assert used == R.ALGO_TREE
    want = R.expected(AR, used, O.FP32, O.SUM, xs, count)
    for r in range(n):
        assert O.equal_bits(O.FP32, outs[r], want[r]), r
    xi = [O.random_operands(O.INT32, count, seed=700 + r, edge=False) for r in range(n)]
    used, _ = collective(comms, AR, 0, O.INT32, O.SUM, xi, count)
    assert used != R.ALGO_TREE


@pytest.mark.parametrize("streams", ["auto", "two"])
@pytest.mark.parametrize("count", [1, 1000, 262147])
@pytest.mark.parametrize("n", [2, 3, 4, 8])
@pytest.mark.parametrize("op_type,algo", CASES)
def test_fp32_sum(worlds, op_type, algo, n, count, streams, monkeypatch):
    """streams: 'auto' runs payloads <= 1 MiB on the caller's stream only; 'two' forces the link/reduce stream
    split with event-derived dependencies at every size."""
    if streams == "two":
        monkeypatch.setenv("HCCL_AMD_SINGLE_STREAM_BYTES", "0")
    comms = worlds(n)
    assert comms[0].get_config(H.Config.SINGLE_STREAM_BYTES) == (0 if streams == "two" else 1 << 20)
    root = n - 1
    in_count = count * n if op_type == RS else count
    xs = [O.random_operands(O.FP32, in_count, seed=31 * n + r, edge=False) for r in range(n)]
    used, outs = collective(comms, op_type, algo, O.FP32, O.SUM, xs, count, root=root, piece_bytes=64 << 10)
    want_ir = oracle_replay(op_type, algo, n, count, O.FP32, O.SUM, xs, root, 64 << 10)
    want_cf = R.expected(op_type, used, O.FP32, O.SUM, xs, count, root=root)
    for r in range(n):
        if op_type == RED and r != root:
            assert not outs[r].any(), "non-root recvBuf written"
            continue
        assert O.equal_bits(O.FP32, outs[r], want_ir[r]), ("vs IR replay", r)
        assert O.equal_bits(O.FP32, outs[r], want_cf[r]), ("vs closed form", r)


def _random_cases(k):
    rng = np.random.default_rng(20261016)
    fams = {AR: [0, 1, 2, 3, 4, 5, 6, 8], RS: [0, 1, 3, 5, 6, 8], RED: [0, 1, 2, 5], AG: [0, 1, 3]}
    dts = [O.INT8, O.INT16, O.INT32, O.INT64, O.UINT64, O.FP16, O.BFP16, O.FP32, O.FP64]
    out = []
    for i in range(k):
        op_type = int(rng.choice([AR, RS, RED, AG]))
        algo = int(rng.choice(fams[op_type]))
        n = int(rng.choice([2, 3, 4, 5, 6, 8]))
        dtype = int(rng.choice(dts))
        op = int(rng.choice(O.OPS)) if op_type != AG else O.SUM
        if op == O.PROD and dtype in (O.INT16, O.BFP16):  # PROD is refused on these (CheckReduceOp)
            op = O.MAX
        count = int(rng.choice([1, 3, 17, 1000, 4099, 65537, 300001]))
        piece = int(rng.choice([0, 4096, 64 << 10]))
        inplace = bool(rng.integers(2)) and op_type == AR
        streams = str(rng.choice(["auto", "two"]))
        out.append((i, op_type, algo, n, dtype, op, count, piece, inplace, streams))
    return out


# HCCL_AMD_RANDOM_DRAWS widens the sweep for a deep one-off run (the default suite takes the first 1000 draws)
@pytest.mark.parametrize("case", _random_cases(int(os.environ.get("HCCL_AMD_RANDOM_DRAWS", "1000"))),
                         ids=lambda c: f"rand{c[0]}")
def test_random_collectives_match_oracle(worlds, monkeypatch, case):
    """Seeded random draws over operation x family x ranks x dtype x op x count x granule x in-place x executor mode
    (combinations the fixed matrices do not pair up), each bit-exact against the oracle replaying the same IR."""
    _, op_type, algo, n, dtype, op, count, piece, inplace, streams = case
    if streams == "two":
        monkeypatch.setenv("HCCL_AMD_SINGLE_STREAM_BYTES", "0")
    comms = worlds(n)
    assert comms[0].get_config(H.Config.SINGLE_STREAM_BYTES) == (0 if streams == "two" else 1 << 20)
    root = (count + n) % n
    in_count = count * n if op_type == RS else count
    xs = [O.random_operands(dtype, in_count, seed=7000 + 13 * case[0] + r, edge=False) for r in range(n)]
    used, outs = collective(comms, op_type, algo, dtype, op, xs, count, root=root, piece_bytes=piece, inplace=inplace)
    want = oracle_replay(op_type, used, n, count, dtype, op, xs, root, piece)
    for r in range(n):
        if op_type == RED and r != root:
            if not inplace:
                assert not outs[r].any(), "non-root recvBuf written"
            continue
        assert O.equal_bits(dtype, outs[r], want[r]), (case, r)


def _random_ipc_cases(k):
    rng = np.random.default_rng(20261017)
    dts = [O.INT8, O.INT16, O.INT32, O.INT64, O.UINT64, O.FP16, O.BFP16, O.FP32, O.FP64]
    out = []
    for i in range(k):
        op_type = int(rng.choice([AR, AR, RS, RED, AG]))
        n = int(rng.choice([2, 3, 4, 8]))
        algo = int(rng.choice([7, 9] + ([12] if op_type == AR and n & (n - 1) == 0 else [])))
        dtype = int(rng.choice(dts))
        op = int(rng.choice(O.OPS)) if op_type != AG else O.SUM
        if op == O.PROD and dtype in (O.INT16, O.BFP16):
            op = O.MAX
        count = int(rng.choice([1, 5, 100, 4099, 65537, 300001, (3 << 20) + 1]))
        out.append((i, op_type, algo, n, dtype, op, count))
    return out


def _ipc_twin(op_type, algo, n, count, dtype, op):
    """The RCCL-path family whose bits an IPC family gives: IPC_TWOSHOT = two-shot AllReduce (O2) / mesh
    ReduceScatter (O1) / two-shot Reduce; IPC = the auto selector's family; IPC_RHD = RHD."""
    if algo == 12:
        return R.ALGO_RHD
    if algo == 7:
        return 1 if op_type in (RS, AG) else 2
    es = np.dtype(O.NP_STORAGE[dtype]).itemsize
    special = dtype in (O.INT64, O.UINT64, O.FP64) or op == O.PROD
    return H.select_algo(op_type, n, count * es, special)


@pytest.mark.parametrize("case", _random_ipc_cases(int(os.environ.get("HCCL_AMD_RANDOM_DRAWS_IPC", "300"))),
                         ids=lambda c: f"ipc{c[0]}")
def test_random_ipc_collectives_match_their_rccl_twin(worlds, monkeypatch, case):
    """Seeded random draws over the one-sided kernel's families (IPC_TWOSHOT, IPC, IPC_RHD) x operation x ranks x
    dtype x op x count, each bit-exact against the oracle replaying the RCCL-path schedule whose order it follows."""
    _, op_type, algo, n, dtype, op, count = case
    monkeypatch.setenv("HCCL_AMD_IPC_TIMEOUT_MS", "20000")
    comms = worlds(n)
    root = (count + 1) % n
    in_count = count * n if op_type == RS else count
    xs = [O.random_operands(dtype, in_count, seed=9100 + 17 * case[0] + r, edge=False) for r in range(n)]
    used, outs = collective(comms, op_type, algo, dtype, op, xs, count, root=root)
    assert used == algo, used
    assert ipc_status(comms[0]) & 1 == 0
    want = oracle_replay(op_type, _ipc_twin(op_type, algo, n, count, dtype, op), n, count, dtype, op, xs, root, 0)
    for r in range(n):
        if op_type == RED and r != root:
            assert not outs[r].any(), "non-root recvBuf written"
            continue
        assert O.equal_bits(dtype, outs[r], want[r]), (case, r)


@pytest.mark.parametrize("dtype", [O.INT8, O.INT16, O.INT32, O.INT64, O.UINT64, O.FP16, O.BFP16, O.FP64],
                         ids=lambda v: O.DTYPE_NAMES[v])
@pytest.mark.parametrize("op", O.OPS, ids=lambda v: O.OP_NAMES[v])
@pytest.mark.parametrize("op_type,algo", [(AR, 1), (AR, 2), (AR, 3), (AR, 4), (AR, 5), (AR, 6), (AR, 7), (AR, 8),
                                          (AR, 9), (RS, 1), (RS, 5), (RS, 6), (RS, 7), (RS, 8), (RS, 9), (RED, 2),
                                          (RED, 5), (RED, 7), (RED, 9)])
def test_dtypes_ops(worlds, op_type, algo, dtype, op):
    n, count, root = 4, 40961, 2
    comms = worlds(n)
    in_count = count * n if op_type == RS else count
    xs = [O.random_operands(dtype, in_count, seed=77 + r, edge=True) for r in range(n)]
    if op == O.PROD and dtype in (O.INT16, O.BFP16):
        # CheckReduceOp (op_common.cc:2977-2998): PROD is not accepted for these dtypes
        with pytest.raises(AssertionError, match="HCCL_E_NOT_SUPPORT"):
            collective(comms, op_type, algo, dtype, op, xs, count, root=root)
        return
    used, outs = collective(comms, op_type, algo, dtype, op, xs, count, root=root, piece_bytes=32 << 10)
    want = oracle_replay(op_type, algo, n, count, dtype, op, xs, root, 32 << 10)
    for r in range(n):
        if op_type == RED and r != root:
            continue
        assert O.equal_bits(dtype, outs[r], want[r]), r


@pytest.mark.parametrize("nbytes", [1 << 10, 64 << 10, 1 << 20, 16 << 20, 64 << 20])
def test_c5_rhd_fp16_random_bit_exact(worlds, nbytes):
    """C5's schedule and dtype (RHD, fp16 SUM, 8 ranks) on random data, where the association order decides the bits:
    bit-exact against the oracle replaying the same IR and against the closed form (n-1 concurrent RHD instances,
    each the classic pairwise halving on its virtual ranks), from 1 KiB to 64 MiB per rank."""
    n, count = 8, nbytes // 2
    comms = worlds(n)
    xs = [O.random_operands(O.FP16, count, seed=900 + r, edge=False) for r in range(n)]
    used, outs = collective(comms, AR, R.ALGO_RHD, O.FP16, O.SUM, xs, count)
    assert used == R.ALGO_RHD
    want_ir = oracle_replay(AR, R.ALGO_RHD, n, count, O.FP16, O.SUM, xs, 0, 0)
    for r in range(n):
        assert O.equal_bits(O.FP16, outs[r], want_ir[r]), ("vs IR replay", r)
    if nbytes <= (1 << 20):  # the numpy closed form is slow at the larger sizes; the IR replay covers them
        want_cf = R.expected(AR, R.ALGO_RHD, O.FP16, O.SUM, xs, count)
        for r in range(n):
            assert O.equal_bits(O.FP16, outs[r], want_cf[r]), ("vs closed form", r)


@pytest.mark.parametrize("n,dtype,op,count", [
    (8, O.FP16, O.SUM, 512), (8, O.FP16, O.SUM, 32 << 10), (8, O.FP16, O.SUM, 1 << 19),
    (8, O.FP16, O.SUM, (1 << 20) + 77),  # 2 MiB: two RHD instances, ragged chunks
    (8, O.FP16, O.SUM, 8 << 20),  # 16 MiB: five instances
    (8, O.FP16, O.SUM, 32 << 20),  # 64 MiB: all seven instances, four staging rounds
    (4, O.FP32, O.SUM, 1000003), (2, O.BFP16, O.SUM, 70001), (8, O.FP32, O.MAX, 300007), (4, O.FP32, O.MIN, 4099),
    (8, O.INT32, O.PROD, 9999), (8, O.FP32, O.SUM, (3 << 20) + 5),
    (8, O.FP32, O.SUM, 7), (4, O.FP16, O.SUM, 1),  # fewer elements than ranks: everything in chunk 0
])
def test_ipc_rhd_is_rhd_bit_exact(worlds, monkeypatch, n, dtype, op, count):
    """HCCL_AMD_ALGO_IPC_RHD: RHD's bits (the RHD schedule's IR replayed by the oracle) from one one-shot launch of the
    one-sided kernel, across one to seven RHD instances, ragged chunks, several staging rounds, the src/dst roles of
    MAX/MIN on ties and NaN (edge operands)."""
    monkeypatch.setenv("HCCL_AMD_IPC_TIMEOUT_MS", "20000")  # a stuck barrier fails the test, never hangs the box
    comms = worlds(n)
    edge = op in (O.MAX, O.MIN)
    xs = [O.random_operands(dtype, count, seed=950 + r, edge=edge) for r in range(n)]
    used, outs = collective(comms, AR, H.Algo.IPC_RHD, dtype, op, xs, count)
    assert used == H.Algo.IPC_RHD
    assert ipc_status(comms[0]) & 1 == 0
    want = oracle_replay(AR, R.ALGO_RHD, n, count, dtype, op, xs, 0, 0)
    for r in range(n):
        assert O.equal_bits(dtype, outs[r], want[r]), r


@pytest.mark.parametrize("n,count", [(8, 300007), (4, (9 << 20) + 1)])
def test_ipc_rhd_in_place(worlds, monkeypatch, n, count):
    """IPC_RHD with sendBuf == recvBuf: every rank pushes a round's elements before it folds over them, so in-place
    keeps RHD's bits (one and several staging rounds)."""
    monkeypatch.setenv("HCCL_AMD_IPC_TIMEOUT_MS", "20000")
    comms = worlds(n)
    xs = [O.random_operands(O.FP32, count, seed=970 + r, edge=False) for r in range(n)]
    used, outs = collective(comms, AR, H.Algo.IPC_RHD, O.FP32, O.SUM, xs, count, inplace=True)
    assert used == H.Algo.IPC_RHD
    want = oracle_replay(AR, R.ALGO_RHD, n, count, O.FP32, O.SUM, xs, 0, 0)
    for r in range(n):
        assert O.equal_bits(O.FP32, outs[r], want[r]), r


def aiv_expected(op_type, dtype, op, xs, count, n, core_limit):
    es = np.dtype(O.NP_STORAGE[dtype]).itemsize
    variant, group = R.aiv_select(op_type, n, count, es, dtype in (O.UINT64, O.FP64), op == O.PROD,
                                  core_limit=core_limit)
    if op_type == AR:
        return variant, R.allreduce_aiv(dtype, op, xs, variant, group)
    return variant, R.reduce_scatter_aiv(dtype, op, xs, count, variant)


# (op, n, count, core limit): every variant of the AIV engine -- one-shot (O2), large-core two-shot (O1 over
# groupSize * n balanced slices; ragged counts put chunk starts off the 16-B grid), small-core two-shot (O2, a core
# limit below 2n blocks), ReduceScatter local tree (O4: small output, or a core limit of at most 2n) and big-data (O2)
AIV_CASES = [(AR, 2, 5001, 48), (AR, 8, 30000, 48), (AR, 4, (1 << 20) + 3, 48), (AR, 8, (1 << 20) + 7, 48),
             (AR, 8, 100003, 48), (AR, 3, 400001, 56), (AR, 8, 70001, 9), (AR, 4, 300007, 8),
             (RS, 4, 1001, 48), (RS, 8, 30001, 48), (RS, 2, (1 << 17) + 5, 48), (RS, 8, (1 << 17) + 1, 48),
             (RS, 8, (1 << 17) + 1, 16), (RS, 3, 200003, 6), (RS, 8, 30001, 4), (AR, 8, 70001, 4)]


@pytest.mark.parametrize("dtype,op", [(O.FP32, O.SUM), (O.FP16, O.SUM), (O.BFP16, O.MAX), (O.INT8, O.SUM),
                                      (O.FP32, O.MIN)], ids=lambda v: str(v))
@pytest.mark.parametrize("op_type,n,count,core_limit", AIV_CASES)
def test_aiv_engine_orders(worlds, monkeypatch, op_type, n, count, core_limit, dtype, op):
    """HCCL_AMD_ALGO_AIV (= HCCL_OP_EXPANSION_MODE=AIV): SelectAivAlgo's variant for the core limit, each folded in
    its kernel's order on the one-sided kernel, bit-exact against the closed forms of tests/sched_ref.py."""
    monkeypatch.setenv("HCCL_AMD_AIV_CORE_LIMIT", str(core_limit))
    comms = worlds(n)
    in_count = count * n if op_type == RS else count
    xs = [O.random_operands(dtype, in_count, seed=1300 + 7 * n + r, edge=False) for r in range(n)]
    variant, want = aiv_expected(op_type, dtype, op, xs, count, n, core_limit)
    assert variant != R.AIV_NOT_MATCHED
    assert int(H.select_aiv_algo(op_type, n, count, dtype, op, core_limit)[0]) == variant
    used, outs = collective(comms, op_type, H.Algo.AIV, dtype, op, xs, count)
    assert used == H.Algo.AIV
    for r in range(n):
        assert O.equal_bits(dtype, outs[r], want[r]), (r, variant)


def _random_aiv_cases(k):
    rng = np.random.default_rng(20261018)
    dts = [O.INT8, O.INT16, O.INT32, O.INT64, O.FP16, O.BFP16, O.FP32]  # the AIV engine's dtypes (no UINT64/FP64)
    out = []
    while len(out) < k:
        op_type = int(rng.choice([AR, RS]))
        n = int(rng.choice([2, 3, 4, 5, 8]))
        dtype = int(rng.choice(dts))
        op = int(rng.choice([O.SUM, O.MAX, O.MIN]))  # PROD is not an AIV op (falls back)
        count = int(rng.choice([1, 7, 1001, 30001, 70001, 131077, 300007, (1 << 20) + 3]))
        core_limit = int(rng.choice([4, 6, 9, 16, 48, 56]))
        es = np.dtype(O.NP_STORAGE[dtype]).itemsize
        variant, _ = R.aiv_select(op_type, n, count, es, False, False, core_limit=core_limit)
        if variant == R.AIV_NOT_MATCHED:
            continue
        out.append((len(out), op_type, n, dtype, op, count, core_limit))
    return out


@pytest.mark.parametrize("case", _random_aiv_cases(int(os.environ.get("HCCL_AMD_RANDOM_DRAWS_AIV", "150"))),
                         ids=lambda c: f"aiv{c[0]}")
def test_random_aiv_engine_orders(worlds, monkeypatch, case):
    """Seeded random draws over the AIV engine (operation x ranks x dtype x op x count x vector-core limit), each
    bit-exact against the closed form of the variant SelectAivAlgo picks."""
    _, op_type, n, dtype, op, count, core_limit = case
    monkeypatch.setenv("HCCL_AMD_AIV_CORE_LIMIT", str(core_limit))
    monkeypatch.setenv("HCCL_AMD_IPC_TIMEOUT_MS", "20000")
    comms = worlds(n)
    in_count = count * n if op_type == RS else count
    xs = [O.random_operands(dtype, in_count, seed=9700 + 11 * case[0] + r, edge=False) for r in range(n)]
    variant, want = aiv_expected(op_type, dtype, op, xs, count, n, core_limit)
    used, outs = collective(comms, op_type, H.Algo.AIV, dtype, op, xs, count)
    assert used == H.Algo.AIV
    for r in range(n):
        assert O.equal_bits(dtype, outs[r], want[r]), (case, r, variant)


@pytest.mark.parametrize("n,count", [(8, (1 << 20) + 7), (4, (3 << 19) + 5), (3, 700001)])
def test_aiv_two_shot_slices_follow_its_loops(monkeypatch, n, count):
    """The AIV large-core two-shot slices every executor loop of min(UB_MAX_DATA_SIZE, ccl/4) into groupSize * n
    balanced slices on its own, so the loop boundaries decide which rank's copy each element's fold starts from. With
    HCCL_BUFFSIZE = 1 MB the loops are 256 KiB: many loops, every one sliced afresh, bit-exact with the closed form."""
    monkeypatch.setenv("HCCL_BUFFSIZE", "1")
    comms = H.loopback_world(n)
    try:
        xs = [O.random_operands(O.FP32, count, seed=1600 + r, edge=False) for r in range(n)]
        variant, want = aiv_expected(AR, O.FP32, O.SUM, xs, count, n, 48)
        assert variant == R.AIV_AR_TWOSHOT_LARGE
        used, outs = collective(comms, AR, H.Algo.AIV, O.FP32, O.SUM, xs, count)
        assert used == H.Algo.AIV
        for r in range(n):
            assert O.equal_bits(O.FP32, outs[r], want[r]), r
    finally:
        torch.cuda.synchronize()
        for c in comms:
            c.destroy()


def test_aiv_expansion_mode_env_and_fallback(worlds, monkeypatch):
    """HCCL_OP_EXPANSION_MODE=AIV on an auto communicator takes the AIV engine; what SelectAivAlgo does not match
    (PROD, FP64, 64 MiB at 8 ranks) runs the AICPU selection, as the reference falls back."""
    monkeypatch.setenv("HCCL_OP_EXPANSION_MODE", "AIV")
    n = 4
    comms = worlds(n)
    xs = [O.random_operands(O.FP32, 3001, seed=1400 + r, edge=False) for r in range(n)]
    used, outs = collective(comms, AR, H.Algo.AUTO, O.FP32, O.SUM, xs, 3001)
    assert used == H.Algo.AIV
    want = R.allreduce_o2(O.FP32, O.SUM, xs)
    for r in range(n):
        assert O.equal_bits(O.FP32, outs[r], want[r]), r
    used, outs = collective(comms, AR, H.Algo.AUTO, O.FP32, O.PROD, xs, 3001)
    assert used == R.ALGO_ONESHOT  # AICPU one-shot (O1)
    want = R.allreduce_o1(O.FP32, O.PROD, xs)
    for r in range(n):
        assert O.equal_bits(O.FP32, outs[r], want[r]), r


def test_aiv_only_has_no_fallback(worlds):
    """HCCL_AMD_ALGO_AIV_ONLY (OpExecuteConfig::AIV_ONLY): the AIV engine above 8 MiB x n as well (64 MiB at 8 ranks
    runs the large-core two-shot, bit-exact), and an operation it does not match (PROD, Reduce) returns
    HCCL_E_NOT_SUPPORT on every rank instead of falling back (op_common.cc:115-122)."""
    n, count = 8, (64 << 20) // 4 + 3
    comms = worlds(n)
    xs = [O.random_operands(O.FP32, count, seed=1500 + r, edge=False) for r in range(n)]
    assert H.select_aiv_algo(AR, n, count, O.FP32, O.SUM)[0] == H.AivVariant.NOT_MATCHED
    variant, group = H.select_aiv_algo(AR, n, count, O.FP32, O.SUM, aiv_only=True)
    assert variant == H.AivVariant.AR_TWOSHOT_LARGE
    used, outs = collective(comms, AR, H.Algo.AIV_ONLY, O.FP32, O.SUM, xs, count)
    assert used == H.Algo.AIV_ONLY
    want = R.allreduce_aiv(O.FP32, O.SUM, xs, int(variant), group)
    for r in range(n):
        assert O.equal_bits(O.FP32, outs[r], want[r]), r
    small = [torch.ones(1024, device="cuda") for _ in range(n)]
    ss = [torch.cuda.Stream() for _ in range(n)]
    for c in comms:
        c.set_algo(H.Algo.AIV_ONLY)
    try:
        for call in (lambda r: comms[r].all_reduce(small[r], small[r], O.PROD, ss[r]),
                     lambda r: comms[r].reduce(small[r], small[r], 0, O.SUM, ss[r])):
            codes = [None] * n

            def body(r, call=call):
                try:
                    call(r)
                    codes[r] = 0
                except H.HcclError as e:
                    codes[r] = e.code

            run_ranks(n, body)
            assert codes == [H.HcclResult.HCCL_E_NOT_SUPPORT] * n, codes
        torch.cuda.synchronize()
        assert all(torch.equal(x, torch.ones_like(x)) for x in small)  # nothing ran
    finally:
        for c in comms:
            c.set_algo(0)


@pytest.mark.parametrize("n,layout", [(2, "ragged"), (4, "gapped"), (8, "ragged"), (8, "overlap"), (3, "empty"),
                                      (4, "empty0")])
@pytest.mark.parametrize("dtype,op", [(O.FP32, O.SUM), (O.FP16, O.SUM), (O.BFP16, O.MAX), (O.INT32, O.PROD),
                                      (O.INT64, O.MIN)], ids=lambda v: str(v))
@pytest.mark.parametrize("streams", ["auto", "two", "ipc"])
def test_reduce_scatter_v(worlds, monkeypatch, n, layout, dtype, op, streams):
    """HcclReduceScatterV through the executor: rank r's output is the mesh template's O1 fold of every rank's block r
    (ins_temp_reduce_scatter_v_mesh_1D.cc:107-146), bit-exact against the closed form and the oracle's IR replay.
    "ipc": the same call on the one-sided kernel over per-rank blocks (kIpcGeomV), the path IPC-only communicators
    take."""
    if streams == "two":
        monkeypatch.setenv("HCCL_AMD_SINGLE_STREAM_BYTES", "0")
    if streams == "ipc":
        monkeypatch.setenv("HCCL_AMD_IPC_TIMEOUT_MS", "20000")
    comms = worlds(n)
    for c in comms:
        c.set_algo(9 if streams == "ipc" else 0)
    if layout == "gapped":
        counts, displs = [70001] * n, [q * 80000 + 3 for q in range(n)]
    elif layout == "overlap":
        counts, displs = [300007] * n, [q * 1000 for q in range(n)]
    elif layout == "empty0":  # rank 0's own block is empty: it must still take part (a loopback world launches
        counts, displs = [0] + [50003] * (n - 1), [0] + [q * 50003 for q in range(n - 1)]  # from rank 0)
    else:
        counts = [(40961 * (q + 3)) % 150001 + (0 if layout != "empty" or q != 1 else -((40961 * 4) % 150001))
                  for q in range(n)]
        displs = list(np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(int))
    in_count = max(c + d for c, d in zip(counts, displs))
    xs = [O.random_operands(dtype, in_count, seed=1500 + r, edge=False) for r in range(n)]
    sends = [to_device(dtype, x) for x in xs]
    recvs = [to_device(dtype, np.zeros(max(1, counts[r]), O.NP_STORAGE[dtype])) for r in range(n)]
    streams_ = [torch.cuda.Stream() for _ in range(n)]
    for c in comms:
        c.set_piece_bytes(64 << 10)
    torch.cuda.synchronize()
    try:
        run_ranks(n, lambda r: comms[r].reduce_scatter_v(sends[r], counts, displs, recvs[r], op, streams_[r]))
        torch.cuda.synchronize()
        used = comms[0].last_algo
    finally:
        for c in comms:
            c.set_piece_bytes(0)
            c.set_algo(0)
    if streams == "ipc":
        assert used == 9 and ipc_status(comms[0]) & 1 == 0
    want = R.reduce_scatter_v_o1(dtype, op, xs, counts, displs)
    for r in range(n):
        got = to_host(dtype, recvs[r])[:counts[r]]
        assert O.equal_bits(dtype, got, want[r]), (r, counts[r])


@pytest.mark.parametrize("algo,nbytes", [(3, (8 << 20) + 28), (3, (58 << 20) + 4), (4, (2 << 20) + 12),
                                         (4, (49 << 19) + 20)])
def test_wide_rings_and_rhd(worlds, algo, nbytes):
    """Ring and RHD on 8 ranks at the sizes where they run several rings / instances at once (2 and 7 rings; 2 and 7
    RHD instances), random fp32: bit-exact against the closed forms of tests/sched_ref.py."""
    n, count = 8, nbytes // 4
    comms = worlds(n)
    xs = [np.random.default_rng(5000 + r).uniform(-1, 1, count).astype(np.float32) for r in range(n)]
    used, outs = collective(comms, AR, algo, O.FP32, O.SUM, xs, count)
    assert used == algo
    want = R.expected(AR, used, O.FP32, O.SUM, xs, count)
    for r in range(n):
        assert O.equal_bits(O.FP32, outs[r], want[r]), r


@pytest.mark.parametrize("algo", [1, 2, 3, 4, 5, 6, 7, 8])
def test_allreduce_inplace(worlds, algo):
    n, count = 4, 300007
    comms = worlds(n)
    xs = [O.random_operands(O.FP32, count, seed=5 + r, edge=False) for r in range(n)]
    used, outs = collective(comms, AR, algo, O.FP32, O.SUM, xs, count, piece_bytes=128 << 10, inplace=True)
    want = R.expected(AR, used, O.FP32, O.SUM, xs, count)
    for r in range(n):
        assert O.equal_bits(O.FP32, outs[r], want[r]), r


def test_default_selection_large_allreduce(worlds):
    """Auto selection at > 8 MiB picks two-shot (reference default) and stays bit-exact with order O2."""
    n, count = 8, (16 << 20) // 4 + 5
    comms = worlds(n)
    xs = [O.random_operands(O.FP32, count, seed=400 + r, edge=False) for r in range(n)]
    used, outs = collective(comms, AR, 0, O.FP32, O.SUM, xs, count)
    assert used == R.ALGO_TWOSHOT
    want = R.expected(AR, used, O.FP32, O.SUM, xs, count)
    for r in range(n):
        assert O.equal_bits(O.FP32, outs[r], want[r]), r


@pytest.mark.parametrize("op_type,n,count", [(AR, 2, (17 << 20) // 4 + 3), (RS, 4, (4 << 20) // 4 + 5)])
def test_default_selection_meshchunk(monkeypatch, op_type, n, count):
    """Auto selection picks MeshChunk where the reference does (AllReduce bytes * 8/n^2 > 32 MiB, ReduceScatter
    recv bytes * (8/n)^2 > 16 MiB) and reproduces its order O6 over several executor loops (HCCL_BUFFSIZE = 4 MB)."""
    monkeypatch.setenv("HCCL_BUFFSIZE", "4")
    comms = H.loopback_world(n)
    try:
        in_count = count * n if op_type == RS else count
        xs = [O.random_operands(O.FP32, in_count, seed=450 + r, edge=False) for r in range(n)]
        used, outs = collective(comms, op_type, 0, O.FP32, O.SUM, xs, count)
        assert used == R.ALGO_MESHCHUNK
        want = R.expected(op_type, used, O.FP32, O.SUM, xs, count)
        for r in range(n):
            assert O.equal_bits(O.FP32, outs[r], want[r]), r
    finally:
        torch.cuda.synchronize()
        for c in comms:
            c.destroy()


def test_reference_st_largest_case_c3_selection(worlds):
    """The reference ST's largest AllReduce (all_reduce_testcase.cc:288-296: 200 MiB + 1, across the CCL buffer) at
    8 ranks and 260 MiB + 148 B per rank: the default selector takes MeshChunk (bytes * 8/64 > 32 MiB, the C3 branch),
    the default HCCL_BUFFSIZE gives three executor loops, and every output bit follows order O6."""
    n, count = 8, (260 << 20) // 4 + 37
    comms = worlds(n)
    xs = [np.random.default_rng(2000 + r).uniform(-1, 1, count).astype(np.float32) for r in range(n)]
    used, outs = collective(comms, AR, 0, O.FP32, O.SUM, xs, count)
    assert used == R.ALGO_MESHCHUNK
    want = R.expected(AR, used, O.FP32, O.SUM, xs, count)
    for r in range(n):
        assert O.equal_bits(O.FP32, outs[r], want[r]), r


def test_reference_sample_known_answer(worlds):
    """examples/02_collectives/01_allreduce: 8 ranks, x_r[i] = i, fp32 SUM -> [0 8 16 ... 56] on every rank;
    04_reduce_scatter: rank r gets 8r; 05_reduce: root 0 gets [0 8 ... 56], others untouched (zeros)."""
    n = 8
    comms = worlds(n)
    xs = [np.arange(8, dtype=np.float32) for _ in range(n)]
    _, outs = collective(comms, AR, 0, O.FP32, O.SUM, xs, 8)
    for r in range(n):
        assert outs[r].tolist() == [0, 8, 16, 24, 32, 40, 48, 56]
    _, outs = collective(comms, RS, 0, O.FP32, O.SUM, xs, 1)
    for r in range(n):
        assert outs[r].tolist() == [8 * r]
    _, outs = collective(comms, RED, 0, O.FP32, O.SUM, xs, 8, root=0)
    assert outs[0].tolist() == [0, 8, 16, 24, 32, 40, 48, 56]
    for r in range(1, n):
        assert outs[r].tolist() == [0] * 8


def test_repeated_calls_reuse_resources(worlds):
    """Back-to-back collectives on the same communicators and streams (event pool, staging reuse)."""
    n, count = 4, 100003
    comms = worlds(n)
    xs = [O.random_operands(O.FP32, count, seed=900 + r, edge=False) for r in range(n)]
    sends = [to_device(O.FP32, x) for x in xs]
    recvs = [torch.empty_like(s) for s in sends]
    streams = [torch.cuda.Stream() for _ in range(n)]
    for c in comms:
        c.set_piece_bytes(16 << 10)
        c.set_algo(2)  # two-shot: every rank holds the same bits, so the MAX pass is the identity
    torch.cuda.synchronize()

    def body(r):
        for _ in range(5):
            comms[r].all_reduce(sends[r], recvs[r], O.SUM, streams[r])
            comms[r].all_reduce(recvs[r], recvs[r], O.MAX, streams[r])

    run_ranks(n, body)
    torch.cuda.synchronize()
    for c in comms:
        c.set_piece_bytes(0)
        c.set_algo(0)
    want = R.expected(AR, comms[0].last_algo, O.FP32, O.SUM, xs, count)[0]
    for r in range(n):
        assert O.equal_bits(O.FP32, to_host(O.FP32, recvs[r]), want)


@pytest.mark.parametrize("algo", [R.ALGO_TWOSHOT, 3, R.ALGO_MESHCHUNK])
@pytest.mark.parametrize("cache", ["1", "0"])
def test_compiled_schedule_cache(worlds, monkeypatch, algo, cache):
    """Repeated calls reuse the compiled schedule and plan (HcclAmdCommCompileStats); a call whose buffers overlap
    differently (in-place after out-of-place, a new buffer pair, another count) still gets a plan for its own overlap,
    so every result stays bit-exact. HCCL_AMD_PLAN_CACHE=0 compiles every call."""
    monkeypatch.setenv("HCCL_AMD_PLAN_CACHE", cache)
    n = 4
    comms = worlds(n)
    counts = [(3 << 20) // 4 + 5, (3 << 20) // 4 + 5, (3 << 20) // 4 + 5, (2 << 20) // 4 + 9, (3 << 20) // 4 + 5]
    inplace = [False, True, False, False, True]
    streams = [torch.cuda.Stream() for _ in range(n)]
    for c in comms:
        c.set_algo(algo)
        c.set_piece_bytes(256 << 10)  # several pieces: the two-stream executor and its plan
    try:
        before = [c.compile_stats() for c in comms]
        for k, (count, ip) in enumerate(zip(counts, inplace)):
            xs = [O.random_operands(O.FP32, count, seed=3000 + 10 * k + r, edge=False) for r in range(n)]
            sends = [to_device(O.FP32, x) for x in xs]
            recvs = [s if ip else torch.zeros_like(s) for s in sends]
            torch.cuda.synchronize()
            run_ranks(n, lambda r: comms[r].all_reduce(sends[r], recvs[r], O.SUM, streams[r]))
            torch.cuda.synchronize()
            want = R.expected(AR, comms[0].last_algo, O.FP32, O.SUM, xs, count)
            for r in range(n):
                assert O.equal_bits(O.FP32, to_host(O.FP32, recvs[r]), want[r]), (k, r)
        for c, (h0, m0) in zip(comms, before):
            h, m = c.compile_stats()
            if cache == "1":
                assert (h - h0, m - m0) == (3, 2)  # counts 0 and 3 compile; calls 1, 2 and 4 reuse
            else:
                assert (h - h0, m - m0) == (0, 5)
    finally:
        torch.cuda.synchronize()
        for c in comms:
            c.set_algo(0)
            c.set_piece_bytes(0)


def test_async_error_does_not_wait_for_a_collective():
    """HcclGetCommAsyncError is lock-free: a watchdog thread gets an answer at once while another thread sits inside a
    collective on the same communicator (here rank 0 waiting in the loopback rendezvous for rank 1)."""
    import time
    comms = H.loopback_world(2)
    try:
        xs = [torch.ones(1 << 20, device="cuda") for _ in range(2)]
        ss = [torch.cuda.Stream() for _ in range(2)]
        for c in comms:
            c.set_algo(R.ALGO_TWOSHOT)
        torch.cuda.synchronize()
        t = threading.Thread(target=lambda: comms[0].all_reduce(xs[0], xs[0], O.SUM, ss[0]))
        t.start()
        time.sleep(0.5)
        assert t.is_alive()  # rank 0 holds its communicator, waiting for rank 1's sends
        t0 = time.perf_counter()
        assert comms[0].async_error() == 0
        assert time.perf_counter() - t0 < 0.1
        comms[1].all_reduce(xs[1], xs[1], O.SUM, ss[1])
        t.join(120)
        assert not t.is_alive()
        torch.cuda.synchronize()
        for x in xs:
            assert torch.equal(x, torch.full_like(x, 2.0))
    finally:
        torch.cuda.synchronize()
        for c in comms:
            c.destroy()


def test_loopback_failure_word_outlives_rank0():
    """A loopback world's IPC launches report timeouts into one word the world owns, so a rank's async-error query
    stays valid after another rank's communicator (rank 0, which issues the world's launch) is destroyed."""
    comms = H.loopback_world(2)
    xs = [torch.ones(4096, device="cuda") for _ in range(2)]
    ss = [torch.cuda.Stream() for _ in range(2)]
    for c in comms:
        c.set_algo(7)  # IPC two-shot: sets up the one-sided path
    torch.cuda.synchronize()
    run_ranks(2, lambda r: comms[r].all_reduce(xs[r], xs[r], O.SUM, ss[r]))
    torch.cuda.synchronize()
    assert comms[0].last_algo == 7
    assert all(torch.equal(x, torch.full_like(x, 2.0)) for x in xs)
    comms[0].destroy()
    assert comms[1].async_error() == 0
    comms[1].destroy()


def test_entry_checks_match_reference(worlds):
    """Validation order and codes of all_reduce_op.cc:23-157, reduce_scatter_op.cc, reduce_op.cc:106-156."""
    comms = worlds(2)
    c = comms[0].handle
    t = torch.zeros(16, device="cuda")
    s = torch.cuda.Stream().cuda_stream
    p = t.data_ptr()
    E = H.HcclResult
    L = H.lib
    FP32, SUM, PROD = H.HcclDataType.FP32, 0, 1
    assert L.HcclAllReduce(p, p, 0, FP32, SUM, None, None) == E.HCCL_SUCCESS          # count 0 first
    assert L.HcclAllReduce(p, p, 16, FP32, SUM, c, None) == E.HCCL_E_PTR              # stream
    assert L.HcclAllReduce(None, p, 16, FP32, SUM, c, s) == E.HCCL_E_PTR
    assert L.HcclAllReduce(p, p, 0x800000000, FP32, SUM, c, s) == E.HCCL_E_PARA      # > SYS_MAX_COUNT
    assert L.HcclAllReduce(p, p, 16, H.HcclDataType.UINT8, SUM, c, s) == E.HCCL_E_NOT_SUPPORT
    assert L.HcclAllReduce(p, p, 16, H.HcclDataType.BFP16, PROD, c, s) == E.HCCL_E_NOT_SUPPORT
    assert L.HcclAllReduce(p, p, 16, H.HcclDataType.INT16, PROD, c, s) == E.HCCL_E_NOT_SUPPORT
    assert L.HcclReduceScatter(p, p, 0, FP32, SUM, None, None) == E.HCCL_SUCCESS
    assert L.HcclReduceScatter(p, None, 8, FP32, SUM, c, s) == E.HCCL_E_PTR
    assert L.HcclReduce(p, p, 0, FP32, SUM, 0, None, None) == E.HCCL_SUCCESS
    assert L.HcclReduce(p, p, 16, FP32, SUM, 0, c, None) == E.HCCL_E_PTR
    assert L.HcclReduce(p, p, 16, FP32, SUM, 2, c, s) == E.HCCL_E_PARA                # root out of range


@pytest.mark.parametrize("algo", [7, 2])  # IPC_TWOSHOT (one kernel on the caller's stream), MESH_TWOSHOT (executor)
def test_calls_on_two_streams_are_ordered(worlds, algo):
    """Two AllReduces of one communicator on two different streams, enqueued back to back with no host wait: they
    share the communicator's staging, so the second must wait for the first (EntryScope, r03). Both results exact."""
    n, count = 4, (6 << 20) + 5
    comms = worlds(n)
    xa = [O.random_operands(O.FP32, count, seed=1300 + r, edge=False) for r in range(n)]
    xb = [O.random_operands(O.FP32, count, seed=1400 + r, edge=False) for r in range(n)]
    da = [to_device(O.FP32, x) for x in xa]
    db = [to_device(O.FP32, x) for x in xb]
    oa = [torch.empty_like(d) for d in da]
    ob = [torch.empty_like(d) for d in db]
    sa = [torch.cuda.Stream() for _ in range(n)]
    sb = [torch.cuda.Stream() for _ in range(n)]
    for c in comms:
        c.set_algo(algo)
    torch.cuda.synchronize()

    def body(r):
        comms[r].all_reduce(da[r], oa[r], O.SUM, sa[r])
        comms[r].all_reduce(db[r], ob[r], O.SUM, sb[r])

    try:
        run_ranks(n, body)
        torch.cuda.synchronize()
    finally:
        for c in comms:
            c.set_algo(0)
    fam = R.ALGO_TWOSHOT
    wa = R.expected(AR, fam, O.FP32, O.SUM, xa, count)
    wb = R.expected(AR, fam, O.FP32, O.SUM, xb, count)
    for r in range(n):
        assert O.equal_bits(O.FP32, to_host(O.FP32, oa[r]), wa[r]), r
        assert O.equal_bits(O.FP32, to_host(O.FP32, ob[r]), wb[r]), r


def test_fold_timing_reports_the_programs_folds():
    """Config.FOLD_TIMING (bench.py's fold_piece row): the executor brackets every fold launch of a program with timing
    events; HcclAmdCommFoldTiming reports as many folds as the plan launches, their algorithmic bytes exactly as the IR
    has them ((operands + 1) x count x size per REDUCE record), durations inside the program's span, and the result
    stays bit-exact. Off, or on the one-sided kernel, there is nothing to report."""
    n, count = 4, (8 << 20) // 4 + 5
    comms = H.loopback_world(n)
    try:
        xs = [O.random_operands(O.FP32, count, seed=5100 + r, edge=False) for r in range(n)]
        with pytest.raises(H.HcclError):
            comms[0].fold_timing()
        for c in comms:
            c.set_config(H.Config.FOLD_TIMING, 1)
        used, outs = collective(comms, AR, R.ALGO_MESHCHUNK, O.FP32, O.SUM, xs, count)
        assert used == R.ALGO_MESHCHUNK
        want = R.expected(AR, used, O.FP32, O.SUM, xs, count)
        for r in range(n):
            assert O.equal_bits(O.FP32, outs[r], want[r]), r
        for r in range(n):
            arr, nops, _, _ = H.build_schedule(AR, R.ALGO_MESHCHUNK, n, r, count, O.FP32)
            ir_bytes = sum((o.nsrc + 1) * o.count * 4 for o in arr[:nops] if o.kind == H.IrKind.REDUCE)
            t = comms[r].fold_timing()
            assert t["fold_bytes"] == ir_bytes, (r, t, ir_bytes)
            assert 0 < t["folds"] <= sum(1 for o in arr[:nops] if o.kind == H.IrKind.REDUCE), t
            assert 0 < t["fold_us"] <= t["span_us"], t
    finally:
        torch.cuda.synchronize()
        for c in comms:
            c.destroy()
