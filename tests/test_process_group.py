"""torch.distributed backend "hccl" (hccl_amd/process_group.py), host side — no GPU.

The GPU half (tests/test_gpu_process_group.py) runs the reference's PyTorch sample through it. Here: registration
under the reference's backend name, the ReduceOp mapping onto HcclReduceOp (and the ops HCCL lacks), the store
all-gather that bootstraps the IPC-only communicator (two processes over a TCPStore), and the argument checks that
run before any GPU call.
"""
import datetime
import multiprocessing as mp

import pytest
import torch
import torch.distributed as dist

import hccl_amd as H
import hccl_amd.process_group as PG


def test_backend_registered_under_the_reference_name():
    # examples/03_ai_framework/01_pytorch/hccl_pytorch_allreduce_test.py:25-27: backend="hccl"
    assert dist.Backend.HCCL == "hccl"
    assert "hccl" in dist.Backend.backend_list
    assert dist.Backend.backend_capability["hccl"] == ["cuda"]


def test_reduce_op_mapping():
    assert PG.hccl_op(dist.ReduceOp.SUM) == H.HcclReduceOp.SUM
    assert PG.hccl_op(dist.ReduceOp.PRODUCT) == H.HcclReduceOp.PROD
    assert PG.hccl_op(dist.ReduceOp.MAX) == H.HcclReduceOp.MAX
    assert PG.hccl_op(dist.ReduceOp.MIN) == H.HcclReduceOp.MIN
    for op in (dist.ReduceOp.AVG, dist.ReduceOp.BAND, dist.ReduceOp.BOR, dist.ReduceOp.BXOR):
        with pytest.raises(ValueError, match="SUM, PRODUCT, MAX and MIN"):
            PG.hccl_op(op)


def _ag_rank(rank, n, port, q):
    store = dist.TCPStore("127.0.0.1", port, is_master=False, timeout=datetime.timedelta(seconds=60))
    ag = PG.StoreAllGather(store, rank, n, "t")
    rounds = [ag(bytes([rank]) * (3 + i)) for i in range(3)]
    q.put((rank, rounds))


def test_store_all_gather_two_processes():
    n = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    # the parent holds the store's server on a port the OS picks (no free-port race with parallel test workers)
    master = dist.TCPStore("127.0.0.1", 0, is_master=True, wait_for_workers=False,
                           timeout=datetime.timedelta(seconds=60))
    port = master.port
    procs = [ctx.Process(target=_ag_rank, args=(r, n, port, q)) for r in range(n)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=30)
    for r in range(n):
        for i, parts in enumerate(got[r]):
            assert parts == [bytes([q]) * (3 + i) for q in range(n)], (r, i)


def test_group_creation_and_host_checks():
    store = dist.HashStore()
    pg = PG._create(store, 0, 1, datetime.timedelta(seconds=30))
    assert isinstance(pg, dist.ProcessGroup)
    assert pg.getBackendName() == "hccl" and pg.rank() == 0 and pg.size() == 1
    opts = dist.AllreduceOptions()
    with pytest.raises(ValueError, match="GPU tensor"):
        pg.allreduce([torch.zeros(4)], opts)
    with pytest.raises(ValueError, match="SUM, PRODUCT, MAX and MIN"):
        opts.reduceOp = dist.ReduceOp.AVG
        pg.allreduce([torch.zeros(4)], opts)
    # two groups made in the same order on every rank get the same, distinct store prefixes
    pg2 = PG._create(store, 0, 1, datetime.timedelta(seconds=30))
    assert pg._prefix != pg2._prefix
    pg.shutdown()  # no communicator yet: nothing to destroy
