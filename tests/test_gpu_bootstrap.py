"""Communicator creation from a rank table (HcclCommInitClusterInfo) and for all local devices (HcclCommInitAll) on
the one-GPU box. A 1-rank table gives a working communicator; a 2-rank table run by two processes on the same GPU
exercises the TCP unique-id exchange end to end: both ranks must hold the same unique id after it
(HcclAmdLastBootstrap digests), and the only failure allowed is RCCL's refusal of two ranks on one device after it."""
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
    os.environ["HCCL_AMD_CONNECT_TIMEOUT_MS"] = "60000"
    try:
        import hccl_amd as H2
        from hccl_amd._lib import HcclError as E
        try:
            c = H2.comm_init_cluster_info(path, rank)
            c.destroy()
            res = "HCCL_SUCCESS"
        except E as e:
            res = str(e)
        stage, digest = H2.last_bootstrap()
        q.put((rank, res, stage, digest))
    except Exception as e:  # noqa: BLE001
        q.put((rank, f"{type(e).__name__}: {e}", -1, 0))


def test_cluster_info_two_ranks_exchange_unique_id(tmp_path):
    """Both ranks must get through the TCP exchange (stage >= 1) holding the same unique id (equal digests). Past it,
    RCCL may refuse two ranks on one device (HCCL_E_PARA): that is the only failure allowed, and only after the
    exchange. A broken exchange leaves stage 0 or different digests and fails here."""
    path = str(tmp_path / "rt2.json")
    _write_table(path, 2, _free_port())
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_cluster_rank, args=(path, r, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        got = {r: (res, stage, digest) for r, res, stage, digest in (q.get(timeout=300) for _ in procs)}
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(2):
        res, stage, digest = got[r]
        assert stage >= 1, f"rank {r} did not complete the unique-id exchange: {got}"
        assert digest != 0
        assert res == "HCCL_SUCCESS" or ("HCCL_E_PARA" in res and stage == 1), got
    assert got[0][2] == got[1][2], f"the ranks hold different unique ids: {got}"


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
