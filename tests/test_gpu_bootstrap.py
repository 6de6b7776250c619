"""Communicator creation from a rank table (HcclCommInitClusterInfo) and for all local devices (HcclCommInitAll) on
the one-GPU box. A 1-rank table gives a working communicator; a 2-rank table run by two processes on the same GPU
exercises the TCP unique-id exchange end to end — both ranks get past it and then RCCL refuses two ranks on one device
(HCCL_E_PARA), which is the expected outcome here (a broken exchange would end in HCCL_E_TIMEOUT / TCP errors)."""
import json
import multiprocessing as mp
import socket

import pytest
import torch

import hccl_amd as H
from hccl_amd._lib import HcclError

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _write_table(path, n, port):
    devs = [{"device_id": "0", "rank_id": str(r), "host_port": str(port)} for r in range(n)]
    table = {"status": "completed", "version": "1.0", "server_count": "1",
             "server_list": [{"server_id": "node_0", "host_ip": "127.0.0.1", "device": devs}]}
    with open(path, "w") as f:
        json.dump(table, f)


def test_cluster_info_single_rank(tmp_path):
    path = str(tmp_path / "rt1.json")
    _write_table(path, 1, _free_port())
    comm = H.comm_init_cluster_info(path, 0)
    try:
        x = torch.arange(1000, dtype=torch.float32, device="cuda")
        y = torch.zeros_like(x)
        s = torch.cuda.Stream()
        torch.cuda.synchronize()
        comm.all_reduce(x, y, H.HcclReduceOp.SUM, stream=s)
        s.synchronize()
        assert torch.equal(x, y)  # SingleRankProc: a copy
    finally:
        comm.destroy()


def _cluster_rank(path, rank, q):
    import os
    os.environ["HCCL_CONNECT_TIMEOUT"] = "120"
    try:
        import hccl_amd as H2
        from hccl_amd._lib import HcclError as E
        try:
            c = H2.comm_init_cluster_info(path, rank)
            c.destroy()
            q.put((rank, "HCCL_SUCCESS"))
        except E as e:
            q.put((rank, str(e)))
    except Exception as e:  # noqa: BLE001
        q.put((rank, f"{type(e).__name__}: {e}"))


def test_cluster_info_two_ranks_exchange_unique_id(tmp_path):
    path = str(tmp_path / "rt2.json")
    _write_table(path, 2, _free_port())
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_cluster_rank, args=(path, r, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        got = dict(q.get(timeout=300) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(2):
        assert "HCCL_SUCCESS" in got[r] or "HCCL_E_PARA" in got[r], got


def test_comm_init_all_one_device():
    comms = H.comm_init_all([0])
    try:
        assert comms[0].last_algo == -1
        x = torch.full((4096,), 3.0, device="cuda")
        y = torch.zeros_like(x)
        s = torch.cuda.Stream()
        torch.cuda.synchronize()
        comms[0].all_reduce(x, y, H.HcclReduceOp.SUM, stream=s)
        s.synchronize()
        assert torch.equal(x, y)
    finally:
        for c in comms:
            c.destroy()


@pytest.mark.parametrize("devices", [[0, 0], [99], [-1]])
def test_comm_init_all_rejects_bad_device_lists(devices):
    with pytest.raises(HcclError, match="HCCL_E_PARA"):
        H.comm_init_all(devices)
