"""Small AllReduces on the one-sided kernel (HCCL_AMD_SMALL_IPC_BYTES, default 1 MiB per rank; ops.cc RunCollective;
VERDICT r04 next #2).

An AllReduce of the auto family or RHD up to the threshold runs as one launch of the one-sided kernel in the same
order family: the auto family's order (one-shot O1 at these sizes, ins_temp_all_reduce_mesh_1D_one_shot.cc:211-226)
or RHD's (the HCCL_AMD_ALGO_IPC_RHD closed form), so the bits are the schedule's. The suite's other
files run with the rule off (conftest) so that they keep checking the schedules themselves at these sizes; here it is
on, as it is by default outside the suite.
"""
import numpy as np
import pytest
import torch

import hccl_amd as H
from oracle import oracle as O
from tests import sched_ref as R
from tests.test_gpu_collectives import AR, RED, RS, collective, ipc_status, oracle_replay, run_ranks
from tests._util import to_device, to_host

pytestmark = pytest.mark.gpu

DEFAULT = 1 << 20


def world(n, small=DEFAULT):
    comms = H.loopback_world(n)
    for c in comms:
        c.set_config(H.Config.SMALL_IPC_BYTES, small)
    return comms


def destroy(comms):
    torch.cuda.synchronize()
    for c in comms:
        c.destroy()


@pytest.mark.parametrize("dtype,op,count", [
    (O.FP16, O.SUM, 512),            # C5's smallest point, 1 KiB
    (O.FP16, O.SUM, (1 << 19)),      # C5 at 1 MiB, the threshold itself
    (O.FP32, O.SUM, 4099),
    (O.BFP16, O.MAX, 65537),
    (O.INT32, O.PROD, 9999),
    (O.FP64, O.SUM, 3001),           # 64-bit: the selector's special case (still one-shot at this size)
    (O.INT8, O.MIN, 1),
], ids=lambda v: str(v))
@pytest.mark.parametrize("n", [2, 3, 4, 8])
def test_small_auto_allreduce_runs_one_sided_with_the_schedule_bits(n, dtype, op, count):
    comms = world(n)
    try:
        xs = [O.random_operands(dtype, count, seed=4400 + 7 * n + r) for r in range(n)]
        used, outs = collective(comms, AR, H.Algo.AUTO, dtype, op, xs, count)
        assert used == H.Algo.IPC, H.Algo(used).name
        assert ipc_status(comms[0]) & 1 == 0
        want = oracle_replay(AR, H.Algo.AUTO, n, count, dtype, op, xs, 0, 0)  # the auto schedule's IR, replayed
        for r in range(n):
            assert O.equal_bits(dtype, outs[r], want[r]), r
    finally:
        destroy(comms)


@pytest.mark.parametrize("count", [512, 4096 + 3, (1 << 19)])
@pytest.mark.parametrize("n", [2, 4, 8])
def test_small_rhd_allreduce_runs_ipc_rhd_with_rhd_bits(n, count):
    """C5's algorithm at its latency end: RHD's bits from one launch (random fp16, where the order decides them)."""
    comms = world(n)
    try:
        xs = [O.random_operands(O.FP16, count, seed=4500 + 7 * n + r, edge=False) for r in range(n)]
        used, outs = collective(comms, AR, H.Algo.RHD, O.FP16, O.SUM, xs, count)
        assert used == H.Algo.IPC_RHD, H.Algo(used).name
        want = oracle_replay(AR, H.Algo.RHD, n, count, O.FP16, O.SUM, xs, 0, 0)
        rank_order = R.allreduce_o2(O.FP16, O.SUM, xs)[0]
        for r in range(n):
            assert O.equal_bits(O.FP16, outs[r], want[r]), r
        if n > 2 and count > 512:  # the check has teeth: the plain rank-order fold differs somewhere
            assert not O.equal_bits(O.FP16, want[0], rank_order)
    finally:
        destroy(comms)


def test_threshold_and_switch():
    """Above the threshold (a ReduceScatter's whole input counted), with the rule off, and for an explicit family the
    schedules run as before."""
    n = 4
    comms = world(n, small=64 << 10)
    try:
        xs = [O.random_operands(O.FP32, 20000, seed=4600 + r) for r in range(n)]  # 80 KB > 64 KiB
        used, outs = collective(comms, AR, H.Algo.AUTO, O.FP32, O.SUM, xs, 20000)
        assert used == R.ALGO_ONESHOT, H.Algo(used).name
        used, _ = collective(comms, AR, H.Algo.AUTO, O.FP32, O.SUM, [x[:1000] for x in xs], 1000)
        assert used == H.Algo.IPC
        # ReduceScatter: 4 blocks of 1000 fp32 (16 KB of input) take the rule, 4 of 5000 (80 KB) the schedule
        used, _ = collective(comms, 1, H.Algo.AUTO, O.FP32, O.SUM, [x[:4000] for x in xs], 1000)
        assert used == H.Algo.IPC, H.Algo(used).name
        used, _ = collective(comms, 1, H.Algo.AUTO, O.FP32, O.SUM, xs, 5000)
        assert used == R.ALGO_ONESHOT, H.Algo(used).name
        # an explicit family is never rerouted
        used, _ = collective(comms, AR, H.Algo.MESH_TWOSHOT, O.FP32, O.SUM, [x[:1000] for x in xs], 1000)
        assert used == R.ALGO_TWOSHOT
        for c in comms:
            c.set_config(H.Config.SMALL_IPC_BYTES, 0)
            assert c.get_config(H.Config.SMALL_IPC_BYTES) == 0
        used, _ = collective(comms, AR, H.Algo.AUTO, O.FP32, O.SUM, [x[:1000] for x in xs], 1000)
        assert used == R.ALGO_ONESHOT
    finally:
        destroy(comms)


def test_in_place_small_allreduce():
    n, count = 4, 3333
    comms = world(n)
    try:
        xs = [O.random_operands(O.FP32, count, seed=4700 + r) for r in range(n)]
        used, outs = collective(comms, AR, H.Algo.AUTO, O.FP32, O.SUM, xs, count, inplace=True)
        assert used == H.Algo.IPC
        want = R.allreduce_o1(O.FP32, O.SUM, xs)
        for r in range(n):
            assert O.equal_bits(O.FP32, outs[r], want[r]), r
    finally:
        destroy(comms)


def test_config_round_trip_and_ranges():
    comms = H.loopback_world(2)
    try:
        c = comms[0]
        assert c.get_config(H.Config.SMALL_IPC_BYTES) == 0  # the suite's environment (conftest)
        assert c.get_config(H.Config.GRAPH_CACHE) == 16
        assert c.get_config(H.Config.IPC_THREADS) == 256
        assert c.get_config(H.Config.IPC_LL_BYTES) == 65536  # the LL form's default
        c.set_config(H.Config.IPC_THREADS, 512)
        assert c.get_config(H.Config.IPC_THREADS) == 512
        for key, bad in ((H.Config.IPC_THREADS, 300), (H.Config.IPC_LIGHT_FENCE, 2), (H.Config.IPC_STAGING_MIB, 8),
                         (H.Config.AIV_CORE_LIMIT, 0), (H.Config.IPC_LL_BYTES, 65537), (H.Config.IPC_LL_BYTES, -1),
                         (99, 1)):
            with pytest.raises(H.HcclError) as e:
                c.set_config(key, bad)
            assert e.value.code == H.HcclResult.HCCL_E_PARA
    finally:
        destroy(comms)


def _random_small_cases(k):
    rng = np.random.default_rng(20261018)
    dts = [O.INT8, O.INT16, O.INT32, O.INT64, O.UINT64, O.FP16, O.BFP16, O.FP32, O.FP64]
    out = []
    for i in range(k):
        n = int(rng.choice([2, 3, 4, 5, 6, 8]))
        algo = int(rng.choice([H.Algo.AUTO, H.Algo.RHD])) if n in (2, 4, 8) else int(H.Algo.AUTO)
        dtype = int(rng.choice(dts))
        op = int(rng.choice(O.OPS))
        if op == O.PROD and dtype in (O.INT16, O.BFP16):  # PROD is refused on these (CheckReduceOp)
            op = O.MAX
        es = np.dtype(O.NP_STORAGE[dtype]).itemsize
        count = int(rng.integers(1, (1 << 20) // es + 1))  # up to the rule's 1 MiB per rank
        inplace = bool(rng.integers(2))
        out.append((i, n, algo, dtype, op, count, inplace))
    return out


@pytest.fixture(scope="module")
def small_worlds():
    cache = {}

    def get(n):
        if n not in cache:
            cache[n] = world(n)
        return cache[n]

    yield get
    torch.cuda.synchronize()
    for comms in cache.values():
        for c in comms:
            c.destroy()


@pytest.mark.parametrize("case", _random_small_cases(200), ids=lambda c: f"small{c[0]}")
def test_random_small_allreduce_matches_the_schedule(small_worlds, case):
    """Seeded draws over ranks x family (auto, RHD) x dtype x op x count (1 .. 1 MiB) x in-place: the one-sided kernel
    the rule picks gives the schedule's bits (the oracle replaying that schedule's IR), edge values included."""
    _, n, algo, dtype, op, count, inplace = case
    comms = small_worlds(n)
    xs = [O.random_operands(dtype, count, seed=12000 + 17 * case[0] + r) for r in range(n)]
    used, outs = collective(comms, AR, algo, dtype, op, xs, count, inplace=inplace)
    assert used == (H.Algo.IPC_RHD if algo == H.Algo.RHD else H.Algo.IPC), H.Algo(used).name
    want = oracle_replay(AR, algo, n, count, dtype, op, xs, 0, 0)
    for r in range(n):
        assert O.equal_bits(dtype, outs[r], want[r]), (case, r)


# ---------------------------------------------------------------------------------------------- the LL form (r05)

LL = 64 << 10


def ll_world(n, ll=LL):
    comms = world(n)
    for c in comms:
        c.set_config(H.Config.IPC_LL_BYTES, ll)
    return comms


def _itemsize(dtype):
    return np.dtype(O.NP_STORAGE[dtype]).itemsize


@pytest.mark.parametrize("dtype,op,count", [
    (O.FP16, O.SUM, 512),           # 1 KiB, C5's smallest point
    (O.INT8, O.MIN, 1),             # one byte: a partial LL word
    (O.INT8, O.SUM, 3),
    (O.INT8, O.MAX, 4101),          # windows whose last word is partial
    (O.FP16, O.SUM, 32767),         # odd fp16 count, just under 64 KiB
    (O.BFP16, O.MAX, 4097),
    (O.FP32, O.SUM, 16384),         # exactly 64 KiB: the largest LL call
    (O.FP32, O.SUM, 16385),         # 4 B over: the staged one-shot
    (O.FP64, O.SUM, 8191),          # 8-byte elements span two LL words
    (O.INT64, O.MAX, 3),
    (O.UINT64, O.SUM, 5),
    (O.INT32, O.PROD, 999),
], ids=lambda v: str(v))
@pytest.mark.parametrize("n", [2, 3, 8])
def test_ll_allreduce_has_the_schedule_bits(n, dtype, op, count):
    """HCCL_AMD_IPC_LL_BYTES: a one-shot AllReduce of at most that many bytes runs in the LL form (data and flag in
    one 8-byte store, no barrier; ipc_kernel_body.h LlOneShot) and gives the auto schedule's bits; one byte over, the
    staged one-shot runs. HcclAmdCommIpcLlLaunches counts the LL launches."""
    comms = ll_world(n)
    try:
        xs = [O.random_operands(dtype, count, seed=5200 + 7 * n + r) for r in range(n)]
        used, outs = collective(comms, AR, H.Algo.AUTO, dtype, op, xs, count)
        assert used == H.Algo.IPC, H.Algo(used).name
        assert comms[0].ipc_ll_launches() == (1 if count * _itemsize(dtype) <= LL else 0)
        assert ipc_status(comms[0]) & 1 == 0
        want = oracle_replay(AR, H.Algo.AUTO, n, count, dtype, op, xs, 0, 0)
        for r in range(n):
            assert O.equal_bits(dtype, outs[r], want[r]), r
    finally:
        destroy(comms)


@pytest.mark.parametrize("count", [1, 512, 4099, 32768])
@pytest.mark.parametrize("n", [2, 4, 8])
def test_ll_rhd_allreduce_has_rhd_bits(n, count):
    """RHD's order from the LL form (IPC_RHD, random fp16 where the order decides the bits)."""
    comms = ll_world(n)
    try:
        xs = [O.random_operands(O.FP16, count, seed=5300 + 7 * n + r, edge=False) for r in range(n)]
        used, outs = collective(comms, AR, H.Algo.RHD, O.FP16, O.SUM, xs, count)
        assert used == H.Algo.IPC_RHD, H.Algo(used).name
        assert comms[0].ipc_ll_launches() == 1
        want = oracle_replay(AR, H.Algo.RHD, n, count, O.FP16, O.SUM, xs, 0, 0)
        for r in range(n):
            assert O.equal_bits(O.FP16, outs[r], want[r]), r
    finally:
        destroy(comms)


def test_ll_calls_back_to_back_with_staged_calls_between():
    """40 AllReduces per rank issued without a host wait: LL calls (both parities, many times over) with a staged
    one-shot (256 KiB) and a two-shot-sized call (4 MiB, the auto family's two-shot) every few calls, fresh random
    inputs per call, each into its own output. Every result has its schedule's bits: the LL flags and parities and
    the staged barrier epochs advance independently and never confuse one call with another."""
    n = 4
    comms = ll_world(n)
    try:
        sizes = []
        for k in range(40):
            sizes.append((4 << 20) // 4 if k % 13 == 12 else (256 << 10) // 4 if k % 5 == 4 else 1 + 97 * k)
        xs = [[O.random_operands(O.FP32, cnt, seed=5400 + 31 * k + r, edge=False) for r in range(n)]
              for k, cnt in enumerate(sizes)]
        sends = [[to_device(O.FP32, xs[k][r]) for r in range(n)] for k in range(len(sizes))]
        recvs = [[torch.empty_like(sends[k][r]) for r in range(n)] for k in range(len(sizes))]
        streams = [torch.cuda.Stream() for _ in range(n)]
        for c in comms:
            c.set_algo(H.Algo.AUTO)
        torch.cuda.synchronize()

        def body(r):
            for k in range(len(sizes)):
                comms[r].all_reduce(sends[k][r], recvs[k][r], O.SUM, streams[r])

        run_ranks(n, body)
        torch.cuda.synchronize()
        assert ipc_status(comms[0]) & 1 == 0
        n_ll = sum(1 for cnt in sizes if cnt * 4 <= LL)
        assert comms[0].ipc_ll_launches() == n_ll
        for k, cnt in enumerate(sizes):
            want = oracle_replay(AR, H.Algo.AUTO, n, cnt, O.FP32, O.SUM, xs[k], 0, 0)
            for r in range(n):
                assert O.equal_bits(O.FP32, to_host(O.FP32, recvs[k][r]), want[r]), (k, cnt, r)
    finally:
        destroy(comms)


def _random_ll_cases(k):
    rng = np.random.default_rng(20261019)
    dts = [O.INT8, O.INT16, O.INT32, O.INT64, O.UINT64, O.FP16, O.BFP16, O.FP32, O.FP64]
    out = []
    for i in range(k):
        n = int(rng.choice([2, 3, 4, 5, 6, 8]))
        algo = int(rng.choice([H.Algo.AUTO, H.Algo.RHD])) if n in (2, 4, 8) else int(H.Algo.AUTO)
        dtype = int(rng.choice(dts))
        op = int(rng.choice(O.OPS))
        if op == O.PROD and dtype in (O.INT16, O.BFP16):
            op = O.MAX
        count = int(rng.integers(1, LL // _itemsize(dtype) + 1))
        out.append((i, n, algo, dtype, op, count, bool(rng.integers(2))))
    return out


@pytest.fixture(scope="module")
def ll_worlds():
    cache = {}

    def get(n):
        if n not in cache:
            cache[n] = ll_world(n)
        return cache[n]

    yield get
    torch.cuda.synchronize()
    for comms in cache.values():
        for c in comms:
            c.destroy()


@pytest.mark.parametrize("case", _random_ll_cases(120), ids=lambda c: f"ll{c[0]}")
def test_random_ll_allreduce_matches_the_schedule(ll_worlds, case):
    """Seeded draws over ranks x family x dtype x op x count (1 .. 64 KiB) x in-place, all in the LL form."""
    _, n, algo, dtype, op, count, inplace = case
    comms = ll_worlds(n)
    before = comms[0].ipc_ll_launches()
    xs = [O.random_operands(dtype, count, seed=13000 + 17 * case[0] + r) for r in range(n)]
    used, outs = collective(comms, AR, algo, dtype, op, xs, count, inplace=inplace)
    assert used == (H.Algo.IPC_RHD if algo == H.Algo.RHD else H.Algo.IPC), H.Algo(used).name
    assert comms[0].ipc_ll_launches() == before + 1
    want = oracle_replay(AR, algo, n, count, dtype, op, xs, 0, 0)
    for r in range(n):
        assert O.equal_bits(dtype, outs[r], want[r]), (case, r)


# ------------------------------------------------------------------ ReduceScatter and Reduce under the rule (r05)

@pytest.mark.parametrize("op_type,n,count,dtype,op", [
    (RS, 2, 5, O.FP32, O.SUM),
    (RS, 4, 4099, O.FP16, O.SUM),
    (RS, 8, 1000, O.BFP16, O.MAX),
    (RS, 3, 8191, O.INT32, O.PROD),
    (RS, 4, (1 << 20) // 16, O.FP32, O.SUM),   # exactly 1 MiB of input per rank: the rule's largest call
    (RED, 2, 5, O.FP32, O.SUM),
    (RED, 4, 40961, O.FP32, O.SUM),
    (RED, 8, 3001, O.FP64, O.MIN),
    (RED, 3, 65537, O.FP16, O.SUM),
], ids=lambda v: str(v))
def test_small_reduce_scatter_and_reduce_run_one_sided(op_type, n, count, dtype, op):
    """The rule takes ReduceScatter and Reduce of the auto family as well (input bytes per rank at most
    HCCL_AMD_SMALL_IPC_BYTES): one launch of the one-sided kernel in the auto family's order, the auto schedule's bits,
    and a Reduce leaves the non-root outputs untouched."""
    comms = world(n)
    try:
        root = n - 1
        in_count = count * n if op_type == RS else count
        xs = [O.random_operands(dtype, in_count, seed=5600 + 7 * n + r) for r in range(n)]
        used, outs = collective(comms, op_type, H.Algo.AUTO, dtype, op, xs, count, root=root)
        assert used == H.Algo.IPC, H.Algo(used).name
        assert ipc_status(comms[0]) & 1 == 0
        want = oracle_replay(op_type, H.Algo.AUTO, n, count, dtype, op, xs, root, 0)
        for r in range(n):
            if op_type == RED and r != root:
                assert not outs[r].any(), "non-root recvBuf written"
                continue
            assert O.equal_bits(dtype, outs[r], want[r]), r
    finally:
        destroy(comms)


def test_small_reduce_scatter_threshold_counts_the_whole_input():
    """A ReduceScatter's input is n blocks: 4 ranks x 65,537 fp32 is 1 MiB + 16 B per rank, over the rule, so the
    schedule runs; one element fewer per block fits."""
    n = 4
    comms = world(n)
    try:
        for count, over in (((1 << 20) // 16 + 1, True), ((1 << 20) // 16, False)):
            xs = [O.random_operands(O.FP32, count * n, seed=5700 + r, edge=False) for r in range(n)]
            used, outs = collective(comms, RS, H.Algo.AUTO, O.FP32, O.SUM, xs, count)
            assert (used != H.Algo.IPC) == over, (count, H.Algo(used).name)
            want = oracle_replay(RS, H.Algo.AUTO, n, count, O.FP32, O.SUM, xs, 0, 0)
            for r in range(n):
                assert O.equal_bits(O.FP32, outs[r], want[r]), (count, r)
    finally:
        destroy(comms)


@pytest.mark.parametrize("dtype,op,count", [
    (O.FP32, O.SUM, 1),
    (O.INT8, O.MAX, 5),             # blocks whose ends fall inside an LL word
    (O.FP16, O.SUM, 4097),
    (O.BFP16, O.MIN, 1023),
    (O.FP32, O.SUM, 16384),         # 64 KiB blocks: the largest LL ReduceScatter
    (O.FP32, O.SUM, 16385),         # 4 B over: staged
    (O.FP64, O.PROD, 777),
], ids=lambda v: str(v))
@pytest.mark.parametrize("n", [2, 3, 8])
def test_ll_reduce_scatter_has_the_schedule_bits(n, dtype, op, count):
    """The ReduceScatter in the LL form (blocks of at most HCCL_AMD_IPC_LL_BYTES): each rank pushes block c to rank c as
    LL words and folds its own block from every peer's, the auto schedule's bits; one block over, the staged kernel."""
    comms = ll_world(n)
    try:
        xs = [O.random_operands(dtype, count * n, seed=5800 + 7 * n + r) for r in range(n)]
        used, outs = collective(comms, RS, H.Algo.AUTO, dtype, op, xs, count)
        assert used == H.Algo.IPC, H.Algo(used).name
        assert comms[0].ipc_ll_launches() == (1 if count * _itemsize(dtype) <= LL else 0)
        assert ipc_status(comms[0]) & 1 == 0
        want = oracle_replay(RS, H.Algo.AUTO, n, count, dtype, op, xs, 0, 0)
        for r in range(n):
            assert O.equal_bits(dtype, outs[r], want[r]), r
    finally:
        destroy(comms)


def test_ll_reduce_scatter_and_allreduce_back_to_back():
    """30 calls per rank without a host wait, LL ReduceScatters and LL AllReduces in turn on one communicator (they
    share the LL sequence and both parities), every result exact."""
    n = 4
    comms = ll_world(n)
    try:
        plan = [(RS if k % 2 else AR, 1 + 211 * k) for k in range(30)]
        xs = [[O.random_operands(O.FP32, cnt * (n if kind == RS else 1), seed=5900 + 31 * k + r, edge=False)
               for r in range(n)] for k, (kind, cnt) in enumerate(plan)]
        sends = [[to_device(O.FP32, xs[k][r]) for r in range(n)] for k in range(len(plan))]
        recvs = [[torch.empty(cnt, device="cuda") for _ in range(n)] for (_, cnt) in plan]
        streams = [torch.cuda.Stream() for _ in range(n)]
        for c in comms:
            c.set_algo(H.Algo.AUTO)
        torch.cuda.synchronize()

        def body(r):
            for k, (kind, _) in enumerate(plan):
                if kind == RS:
                    comms[r].reduce_scatter(sends[k][r], recvs[k][r], O.SUM, streams[r])
                else:
                    comms[r].all_reduce(sends[k][r], recvs[k][r], O.SUM, streams[r])

        run_ranks(n, body)
        torch.cuda.synchronize()
        assert ipc_status(comms[0]) & 1 == 0
        assert comms[0].ipc_ll_launches() == len(plan)
        for k, (kind, cnt) in enumerate(plan):
            want = oracle_replay(kind, H.Algo.AUTO, n, cnt, O.FP32, O.SUM, xs[k], 0, 0)
            for r in range(n):
                assert O.equal_bits(O.FP32, to_host(O.FP32, recvs[k][r]), want[r]), (k, kind, cnt, r)
    finally:
        destroy(comms)
