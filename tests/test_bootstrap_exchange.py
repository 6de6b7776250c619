"""The rank-table unique-id exchange of HcclCommInitClusterInfo, host only (no GPU): rank 0 serves the id over TCP and
every other rank must receive exactly rank 0's bytes (the reference's ST builds its communicators from such a table,
test/st/algorithm/testcase/all_reduce_testcase.cc:80). The negative controls show the exchange can fail: a table whose
root never starts ends in HCCL_E_TIMEOUT at the (test-shortened) connect bound, and a rank outside the table is
HCCL_E_PARA."""
import json
import multiprocessing as mp
import os
import socket
import time

import pytest

import hccl_amd as H
from hccl_amd._lib import HcclError


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


def _rank(path, rank, ident, q, env):
    os.environ.update(env)
    try:
        import hccl_amd as H2
        got = H2.bootstrap_exchange_id(path, rank, ident)
        q.put((rank, "ok", got))
    except Exception as e:  # noqa: BLE001
        q.put((rank, str(e), b""))


def _run(path, ranks, ident, env, wait=60):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(path, r, ident if r == 0 else b"", q, env)) for r in ranks]
    for p in procs:
        p.start()
    try:
        got = {}
        for _ in procs:
            r, status, data = q.get(timeout=wait)
            got[r] = (status, data)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return got


@pytest.mark.parametrize("n", [2, 4])
def test_every_rank_receives_rank0_id(tmp_path, n):
    path = str(tmp_path / "rt.json")
    _write_table(path, n, _free_port())
    ident = os.urandom(128)
    got = _run(path, range(n), ident, {})
    for r in range(n):
        assert got[r][0] == "ok", got[r]
        assert got[r][1] == ident, f"rank {r} received other bytes than rank 0 served"


def test_missing_root_times_out(tmp_path):
    path = str(tmp_path / "rt.json")
    _write_table(path, 2, _free_port())
    t0 = time.time()
    got = _run(path, [1], b"", {"HCCL_AMD_CONNECT_TIMEOUT_MS": "1500"})
    assert "HCCL_E_TIMEOUT" in got[1][0], got
    assert time.time() - t0 < 30


def test_rank_outside_table_is_para(tmp_path):
    path = str(tmp_path / "rt.json")
    _write_table(path, 2, _free_port())
    with pytest.raises(HcclError, match="HCCL_E_PARA"):
        H.bootstrap_exchange_id(path, 5, b"")
