"""The library's device memory per communicator: bounded by the reference's buffer
contract and reported exactly by HcclAmdCommDeviceBytes.

The reference keeps 2 x HCCL_BUFFSIZE per communicator (HCCL_BUFFSIZE.md; aiv_defines.h:44). Here:
  * the executor's staging (2 x HCCL_BUFFSIZE) is allocated by the first collective that runs a schedule;
  * the one-sided kernel's base allocations (flags + LL area, status words, LL unpack area) by its first call;
  * its small staging tier (four areas of n x HCCL_AMD_SMALL_IPC_BYTES) by the first call whose staging fits one round
    there, its large tier (four areas of HCCL_BUFFSIZE / 2, or HCCL_AMD_IPC_STAGING_MIB) by the first call that needs
    more.
So a communicator whose calls are all small holds MiBs. The expected byte counts below restate ipc.h's sizes."""
import numpy as np
import pytest
import torch

import hccl_amd as H
from oracle import oracle as O
from tests.test_gpu_collectives import AR, RED, RS, collective

pytestmark = pytest.mark.gpu

MIB = 1 << 20
KIB = 1 << 10
# ipc.h: kIpcFlagBytes (512 blocks x 16 ranks x 4 B) + two LL parities (16 slots x 128 KiB), the status words, the
# unpack area (16 x (64 KiB + 256 B))
BASE_BYTES = 512 * 16 * 4 + 2 * 16 * 128 * KIB + 32 + 16 * (64 * KIB + 256)


def _up64k(b):
    return (b + 64 * KIB - 1) // (64 * KIB) * (64 * KIB)


def small_tier_bytes(n, small=MIB):
    return 4 * _up64k(n * max(small, 64 * KIB))


def large_tier_bytes(area):
    alt = min(area, ((2047 * MIB - 2 * area) // 2) // (64 * KIB) * (64 * KIB))
    return 2 * area + 2 * alt


def _ints(n, count, dtype=O.FP32):
    # integer-valued operands: every order gives the same sum, so a wrong byte is a wrong result
    return [np.full(count, r + 1, O.NP_STORAGE[dtype]) if dtype != O.FP32 else
            (np.arange(count) % 97 + r).astype(np.float32) for r in range(n)]


def test_small_calls_hold_megabytes_and_the_query_is_exact(monkeypatch):
    """A loopback world whose calls are all at most 1 MiB per rank (the small-call rule on, its default): AllReduce,
    ReduceScatter and Reduce of the auto family, 1 KiB to 1 MiB. Every rank then holds exactly the base allocations plus
    the small tier (no executor staging, no large tier): 21 MiB at n = 4, at most 64 MiB."""
    monkeypatch.setenv("HCCL_AMD_SMALL_IPC_BYTES", str(MIB))
    n = 4
    comms = H.loopback_world(n)
    try:
        assert [c.device_bytes() for c in comms] == [0] * n  # nothing until a call needs it
        for op_type, count in ((AR, 256), (AR, MIB // 4), (RS, MIB // 4 // n), (RED, 16 * KIB), (AR, 4099)):
            in_count = count * n if op_type == RS else count
            xs = _ints(n, in_count)
            used, outs = collective(comms, op_type, H.Algo.AUTO, O.FP32, O.SUM, xs, count, root=1)
            assert used == H.Algo.IPC, (op_type, count, H.Algo(used).name)
            total = sum(xs)
            for r in range(n):
                if op_type == RED and r != 1:
                    continue
                want = total[r * count:(r + 1) * count] if op_type == RS else total
                assert np.array_equal(outs[r], want), (op_type, count, r)
        want_bytes = BASE_BYTES + small_tier_bytes(n)
        for c in comms:
            assert c.scratch()[0] == 0, "no schedule ran: no executor staging"
            assert c.device_bytes() == want_bytes, (c.device_bytes(), want_bytes)
            assert c.device_bytes() <= 64 * MIB
    finally:
        torch.cuda.synchronize()
        for c in comms:
            c.destroy()


def test_tiers_and_staging_appear_when_a_call_needs_them(monkeypatch):
    """The same world then runs a schedule (the executor staging appears: 2 x HCCL_BUFFSIZE) and a one-sided call too
    large for the small tier (the large tier appears: four areas of HCCL_AMD_IPC_STAGING_MIB, 128 MiB in the suite),
    each exact; the query follows every step."""
    monkeypatch.setenv("HCCL_AMD_SMALL_IPC_BYTES", str(MIB))
    monkeypatch.setenv("HCCL_BUFFSIZE", "8")
    monkeypatch.setenv("HCCL_AMD_IPC_STAGING_MIB", "32")
    n = 4
    comms = H.loopback_world(n)
    try:
        count = 100000  # above the LL form's 64 KiB: a staged call in the small tier
        xs = _ints(n, count)
        used, outs = collective(comms, AR, H.Algo.AUTO, O.FP32, O.SUM, xs, count)
        assert used == H.Algo.IPC
        assert all(np.array_equal(o, sum(xs)) for o in outs)
        small = BASE_BYTES + small_tier_bytes(n)
        assert [c.device_bytes() for c in comms] == [small] * n
        # a ring AllReduce: the executor staging of 2 x 8 MB
        count = (4 * MIB) // 4
        xs = _ints(n, count)
        used, outs = collective(comms, AR, H.Algo.RING, O.FP32, O.SUM, xs, count)
        assert used == H.Algo.RING
        assert all(np.array_equal(o, sum(xs)) for o in outs)
        assert [c.device_bytes() for c in comms] == [small + 2 * 8 * MIB] * n
        # a two-shot one-sided AllReduce of 16 MiB per rank: chunks of 4 MiB do not fit the small tier's 1 MiB slots
        count = (16 * MIB) // 4 + 5
        xs = _ints(n, count)
        used, outs = collective(comms, AR, H.Algo.IPC_TWOSHOT, O.FP32, O.SUM, xs, count)
        assert used == H.Algo.IPC_TWOSHOT
        assert all(np.array_equal(o, sum(xs)) for o in outs)
        assert [c.device_bytes() for c in comms] == [small + 2 * 8 * MIB + large_tier_bytes(32 * MIB)] * n
        # a small call afterwards still runs exact (from the small tier, whose epochs continue)
        count = 1000
        xs = _ints(n, count)
        used, outs = collective(comms, AR, H.Algo.IPC_TWOSHOT, O.FP32, O.SUM, xs, count)
        assert all(np.array_equal(o, sum(xs)) for o in outs)
    finally:
        torch.cuda.synchronize()
        for c in comms:
            c.destroy()


def test_large_tier_defaults_to_the_reference_buffer_contract(monkeypatch):
    """Without HCCL_AMD_IPC_STAGING_MIB the large tier's areas are HCCL_BUFFSIZE / 2: its four areas hold
    2 x HCCL_BUFFSIZE (here HCCL_BUFFSIZE = 64 MB, so 128 MiB)."""
    monkeypatch.setenv("HCCL_BUFFSIZE", "64")
    monkeypatch.delenv("HCCL_AMD_IPC_STAGING_MIB", raising=False)
    n = 2
    comms = H.loopback_world(n)
    try:
        count = (48 * MIB) // 4 + 3
        xs = _ints(n, count)
        used, outs = collective(comms, AR, H.Algo.IPC_TWOSHOT, O.FP32, O.SUM, xs, count)
        assert used == H.Algo.IPC_TWOSHOT
        assert all(np.array_equal(o, sum(xs)) for o in outs)
        want = BASE_BYTES + large_tier_bytes(32 * MIB)  # the call skipped the small tier: it never fit one round there
        assert [c.device_bytes() for c in comms] == [want] * n
        assert want < 2 * 64 * MIB + 8 * MIB
    finally:
        torch.cuda.synchronize()
        for c in comms:
            c.destroy()


@pytest.mark.parametrize("op_type,count", [(AR, 4099), (AR, (1 << 20) // 4), (RS, 1000), (RED, 5000)])
def test_failed_ipc_allocation_falls_back_to_the_schedule(monkeypatch, op_type, count):
    """when one rank's one-sided set-up cannot allocate, every rank agrees on HCCL_E_NOT_SUPPORT and the
    small-call rule runs the schedule of the same family instead, on every rank alike: the call succeeds with the
    schedule's bits (integer-valued data, so any order is exact) and nothing of the one-sided path is left allocated."""
    monkeypatch.setenv("HCCL_AMD_SMALL_IPC_BYTES", str(MIB))
    monkeypatch.setenv("HCCL_AMD_INJECT_IPC_ALLOC_FAIL", "2")
    n = 4
    comms = H.loopback_world(n)
    try:
        in_count = count * n if op_type == RS else count
        xs = _ints(n, in_count)
        used, outs = collective(comms, op_type, H.Algo.AUTO, O.FP32, O.SUM, xs, count, root=1)
        assert not H.Algo(used).name.startswith("IPC"), H.Algo(used).name
        total = sum(xs)
        for r in range(n):
            if op_type == RED and r != 1:
                continue
            want = total[r * count:(r + 1) * count] if op_type == RS else total
            assert np.array_equal(outs[r], want), r
        for c in comms:
            assert c.device_bytes() == c.scratch()[1], "only the executor staging is held"
        # a later small call takes the schedule at once (the one-sided path stays unavailable, on every rank)
        used, outs = collective(comms, op_type, H.Algo.AUTO, O.FP32, O.SUM, xs, count, root=1)
        assert not H.Algo(used).name.startswith("IPC")
    finally:
        torch.cuda.synchronize()
        for c in comms:
            c.destroy()


_IDLE_CHILD = r'''
import ctypes, os, sys, json
sys.path.insert(0, os.getcwd())
import numpy as np, torch
import hccl_amd as H
from oracle import oracle as O
from tests.test_gpu_collectives import AR, collective
torch.cuda.set_device(0)
out = {"idle_before": H.ipc_idle_staging()}
xs = [(np.arange(100000) % 97 + r).astype(np.float32) for r in range(2)]
exact = True
for k in range(2):
    comms = H.loopback_world(2)
    used, outs = collective(comms, AR, H.Algo.IPC_TWOSHOT, O.FP32, O.SUM, xs, 100000)
    exact = exact and all(np.array_equal(o, xs[0] + xs[1]) for o in outs)
    out[f"idle_while_alive_{k}"] = H.ipc_idle_staging()
    torch.cuda.synchronize()
    for c in comms:
        c.destroy()
    out[f"idle_after_destroy_{k}"] = H.ipc_idle_staging()
b = ctypes.c_uint64(0)
out["release_rc"] = H.lib.HcclAmdIpcIdleStaging(1, ctypes.byref(b))
out["release_reported"] = b.value
out["idle_after_release"] = H.ipc_idle_staging()
out["exact"] = bool(exact)
print(json.dumps(out))
'''


def test_idle_staging_is_reported_and_reused_never_freed():
    """HcclAmdIpcIdleStaging: a destroyed communicator's uncached blocks stay with the process (reported), the next
    communicator's set-up of the same sizes takes them back (the idle total returns to 0 while it lives), and a request
    to release them is refused (HCCL_E_NOT_SUPPORT) after reporting: freeing uncached memory corrupts later GPU work on
    this stack. In a child process, so that the counts start from zero."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _IDLE_CHILD], cwd=root, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["idle_before"] == 0 and out["idle_while_alive_0"] == 0, out
    idle = out["idle_after_destroy_0"]
    assert idle > 0, out
    assert out["idle_while_alive_1"] == 0, out  # the second world's set-up reused every block
    assert out["idle_after_destroy_1"] == idle, out
    assert out["release_rc"] == int(H.HcclResult.HCCL_E_NOT_SUPPORT) and out["release_reported"] == idle, out
    assert out["idle_after_release"] == idle and out["exact"], out
