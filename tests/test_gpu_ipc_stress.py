"""Randomised sequence of IPC collectives in rank mode (n processes sharing the GPU, peers mapped through IPC
handles): every kind (AllReduce one-shot / two-shot / MeshChunk, ReduceScatter, Reduce, AllGather), counts from 1
element to several staging rounds, block counts changing from call to call (default or forced 1..256), order
families fixed (IPC_TWOSHOT), the auto family (IPC) or RHD's order (IPC_RHD). This drives the barrier epochs, the alternating slot areas of
the single-barrier kinds and the per-launch windows through mixes no hand-written case lists.

Data are small integers in fp32, so every association order gives the exact sum and the expected output is a
formula of (call, rank, element), checked on the GPU. The bit-exact order of each family is pinned elsewhere
(test_gpu_ipc_ranks.py, test_gpu_collectives.py); this test is about the protocol."""
import datetime
import multiprocessing as mp
import os
import random
import socket
import time
import traceback

import pytest

pytestmark = pytest.mark.gpu

AR, RS, RED, AG = 0, 1, 2, 3
CALLS = 120
SEED = 20261016


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _plan(n):
    """The call sequence, equal on every rank (same seed)."""
    rng = random.Random(SEED + n)
    sizes = [1, 5, 97, 4099, 65537, 300007, (1 << 20) + 3, (5 << 20) + 1, (9 << 20) + 7]
    plan = []
    for i in range(CALLS):
        kind = rng.choice((AR, AR, RS, RED, AG))
        count = rng.choice(sizes)
        if kind in (RS, AG) and count > (3 << 20):
            count //= n  # keep n x count within a few tens of MiB
        algo = rng.choice((7, 9, 9, 12))  # 12 = IPC_RHD (AllReduce; the other kinds take the auto family)
        blocks = rng.choice((0, 0, 0, 1, 16, 64, 256, rng.randint(1, 256)))
        plan.append((kind, count, algo, blocks, rng.randrange(n)))
    return plan


def _rank_main(rank, n, port, q):
    os.environ["HCCL_AMD_IPC_TIMEOUT_MS"] = "20000"
    os.makedirs("gpurun_out", exist_ok=True)
    progress = open(f"gpurun_out/ipc_stress_n{n}_r{rank}.log", "w", buffering=1)
    try:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=n,
                                timeout=datetime.timedelta(seconds=120))
        torch.cuda.set_device(0)
        import hccl_amd as H

        def all_gather(b):
            out = [None] * n
            dist.all_gather_object(out, b)
            return out

        comm = H.comm_init_host_exchange(n, rank, all_gather)
        stream = torch.cuda.Stream()
        bad = []
        for i, (kind, count, algo, blocks, root) in enumerate(_plan(n)):
            comm.set_algo(algo)
            comm.set_ipc_blocks(blocks)
            in_count = count * n if kind == RS else count
            idx = torch.arange(in_count, device="cuda", dtype=torch.int64)
            send = ((idx * 7 + i) % 113 + rank).to(torch.float32)
            out_count = count * n if kind == AG else count
            recv = torch.full((out_count,), -1.0, device="cuda")
            torch.cuda.synchronize()
            if kind == AR:
                comm.all_reduce(send, recv, H.HcclReduceOp.SUM, stream=stream)
            elif kind == RS:
                comm.reduce_scatter(send, recv, H.HcclReduceOp.SUM, stream=stream)
            elif kind == RED:
                comm.reduce(send, recv, root, H.HcclReduceOp.SUM, stream=stream)
            else:
                comm.all_gather(send, recv, stream=stream)
            stream.synchronize()
            tri = n * (n - 1) // 2
            if kind == AG:
                j = torch.arange(out_count, device="cuda", dtype=torch.int64)
                want = ((j % count * 7 + i) % 113 + j // count).to(torch.float32)
            elif kind == RS:
                g = torch.arange(rank * count, (rank + 1) * count, device="cuda", dtype=torch.int64)
                want = ((g * 7 + i) % 113 * n + tri).to(torch.float32)
            elif kind == RED and rank != root:
                want = torch.full((out_count,), -1.0, device="cuda")  # a non-root recvBuf is never written
            else:
                want = ((idx * 7 + i) % 113 * n + tri).to(torch.float32)
            ok = bool(torch.equal(recv, want))
            status = comm.ipc_status()
            progress.write(f"call {i} kind {kind} count {count} algo {algo} blocks {blocks} ok {ok} "
                           f"status {status:#x}\n")
            if not ok or status & 1:
                bad.append((i, kind, count, algo, blocks, ok, status))
            if max(all_gather(status & 1)) != 0:
                break
        dist.barrier()
        comm.destroy()
        dist.destroy_process_group()
        q.put((rank, "ok", bad))
    except Exception:  # noqa: BLE001
        progress.write(traceback.format_exc())
        q.put((rank, traceback.format_exc(), None))
        time.sleep(10)


@pytest.mark.parametrize("n", [2, 4])
def test_ipc_random_call_sequence(n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, n, port, q)) for r in range(n)]
    for p in procs:
        p.start()
    try:
        got = {}
        for _ in procs:
            rank, msg, res = q.get(timeout=300)
            got[rank] = (msg, res)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(n):
        assert got[r][0] == "ok", f"rank {r}:\n{got[r][0]}"
        assert got[r][1] == [], f"rank {r}: {got[r][1][:5]}"
