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
    # the keys live under a fixed prefix of the store torch gives each group (a PrefixStore on the group name)
    pg2 = PG._create(store, 0, 1, datetime.timedelta(seconds=30))
    assert pg._prefix == pg2._prefix == "hccl_amd"
    pg.shutdown()  # no communicator yet: nothing to destroy


def _subgroup_rank(rank, n, port, q):
    """Overlapping subgroups ([0, 1] then [1, 2]) over the "hccl" backend: each subgroup's bootstrap key must be the
    same on its members, although rank 0 and rank 2 each build only one of the two backends (a per-process
    counter had rank 1 and rank 2 disagree on the second group's key, and its first collective hung)."""
    import os
    os.environ["HCCL_AMD_PG_TRANSPORT"] = ""
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=n,
                                timeout=datetime.timedelta(seconds=60))
        blobs = {}

        def fake_root_info():
            return f"root-of-{rank}".encode()

        def fake_init(size, blob, r):
            blobs[len(blobs)] = (size, bytes(blob), r)
            return object()

        H.get_root_info, H.comm_init_root_info = fake_root_info, fake_init
        got = {}
        for members in ([0, 1], [1, 2]):
            g = dist.new_group(members, backend="hccl")
            if rank in members:
                # a ProcessGroup subclass is the group itself (torch's _new_process_group_helper)
                be = g if isinstance(g, PG.ProcessGroupHCCL) else g._get_backend(torch.device("cuda"))
                be._factory(0)  # the bootstrap: the group's rank 0 publishes, every member reads
                got[tuple(members)] = blobs[len(blobs) - 1]
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, got))
    except Exception as e:  # noqa: BLE001
        q.put((rank, f"{type(e).__name__}: {e}"))


def test_overlapping_subgroups_agree_on_the_bootstrap_key():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_subgroup_rank, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    try:
        got = dict(q.get(timeout=120) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(3):
        assert isinstance(got[r], dict), got
    # group [0, 1]: group rank 0 is global rank 0; group [1, 2]: group rank 0 is global rank 1
    assert got[0][(0, 1)] == (2, b"root-of-0", 0) and got[1][(0, 1)] == (2, b"root-of-0", 1)
    assert got[1][(1, 2)] == (2, b"root-of-1", 0) and got[2][(1, 2)] == (2, b"root-of-1", 1)
