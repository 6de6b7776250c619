"""The reference's PyTorch caller through the "hccl" torch.distributed backend (hccl_amd/process_group.py).

examples/03_ai_framework/01_pytorch/hccl_pytorch_allreduce_test.py:19-38 spawns one process per device, calls
``dist.init_process_group(backend="hccl")`` and ``dist.all_reduce`` on ``torch.arange(world_size, float32)``; every
rank must end with ``world_size * arange(world_size)`` (examples/02_collectives/01_allreduce/README_en.md:59-70 for
8 ranks). Here the same body runs with its device calls changed (npu -> cuda):

* world 1 over the RCCL transport, the root-info blob carried by the process group's store;
* worlds 2 and 4 as separate processes sharing the one GPU over the IPC-only communicator
  (HCCL_AMD_PG_TRANSPORT=ipc; RCCL refuses two ranks on one device), with the other collectives the backend maps
  (reduce, reduce_scatter_tensor / list, all_gather_into_tensor / list, barrier, async work) checked exactly, and a
  random fp32 all_reduce checked bit-exact against the reference's one-shot order O1 for its size
  (ins_temp_all_reduce_mesh_1D_one_shot.cc:211-226: acc = x_me, then x_r for r ascending, r != me).
"""
import datetime
import multiprocessing as mp
import os
import socket
import time
import traceback

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, n, port, transport, q):
    os.environ["HCCL_AMD_IPC_TIMEOUT_MS"] = "20000"
    if transport:
        os.environ["HCCL_AMD_PG_TRANSPORT"] = transport
    os.makedirs("gpurun_out", exist_ok=True)
    progress = open(f"gpurun_out/process_group_n{n}_r{rank}.log", "w", buffering=1)
    try:
        import torch
        import torch.distributed as dist
        import hccl_amd.process_group  # noqa: F401  (registers backend "hccl")

        torch.cuda.set_device(0)  # the sample: torch_npu.npu.set_device(rank); one GPU here
        dist.init_process_group(backend="hccl", rank=rank, world_size=n, init_method=f"tcp://127.0.0.1:{port}",
                                timeout=datetime.timedelta(seconds=120))
        checks = {}
        # --- the reference sample's body
        t = torch.arange(n, dtype=torch.float32, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        checks["sample_all_reduce"] = t.cpu().tolist() == [float(n * i) for i in range(n)]
        progress.write(f"sample {t.cpu().tolist()}\n")
        # --- random fp32 all_reduce, bit-exact against order O1 (one-shot at this size)
        count = 4099
        g = np.random.default_rng(1234)
        xs = [g.uniform(-1, 1, count).astype(np.float32) for _ in range(n)]
        x = torch.from_numpy(xs[rank]).cuda()
        dist.all_reduce(x)
        acc = xs[rank].copy()
        for r in range(n):
            if r != rank:
                acc = (xs[r] + acc).astype(np.float32)
        checks["o1_bits"] = np.array_equal(x.cpu().numpy().view(np.uint32), acc.view(np.uint32))
        # --- MAX / MIN / PRODUCT on integers
        v = torch.full((1000,), rank + 2, dtype=torch.int32, device="cuda")
        for op, want in ((dist.ReduceOp.MAX, n + 1), (dist.ReduceOp.MIN, 2),
                         (dist.ReduceOp.PRODUCT, int(np.prod(np.arange(2, n + 2))))):
            y = v.clone()
            dist.all_reduce(y, op=op)
            checks[f"op_{op}"] = bool(torch.all(y == want).item())
        # --- reduce to root 1 % n
        root = 1 % n
        y = torch.full((5001,), float(rank + 1), device="cuda")
        dist.reduce(y, dst=root)
        checks["reduce"] = (not rank == root) or bool(torch.all(y == n * (n + 1) / 2).item())
        # --- reduce_scatter_tensor and the list form
        rc = 3001
        inp = torch.arange(n * rc, dtype=torch.float32, device="cuda") % 113 + rank
        out = torch.empty(rc, device="cuda")
        dist.reduce_scatter_tensor(out, inp)
        want = n * (torch.arange(rank * rc, (rank + 1) * rc, device="cuda", dtype=torch.float32) % 113) + n * (n - 1) / 2
        checks["reduce_scatter_tensor"] = bool(torch.equal(out, want))
        out2 = torch.empty(rc, device="cuda")
        dist.reduce_scatter(out2, list(inp.chunk(n)))
        checks["reduce_scatter_list"] = bool(torch.equal(out2, want))
        # --- reduce_scatter with uneven blocks (HcclReduceScatterV): rank q's block has 1000 + 37 q elements
        sizes = [1000 + 37 * q for q in range(n)]
        blocks = [torch.arange(sz, dtype=torch.float32, device="cuda") % 7 + rank for sz in sizes]
        mine = torch.empty(sizes[rank], device="cuda")
        dist.reduce_scatter(mine, blocks)
        checks["reduce_scatter_uneven"] = bool(torch.equal(
            mine, n * (torch.arange(sizes[rank], dtype=torch.float32, device="cuda") % 7) + n * (n - 1) / 2))
        # --- all_gather_into_tensor and the list form (bf16: data movement, any dtype)
        a = torch.full((777,), float(rank), dtype=torch.bfloat16, device="cuda")
        full = torch.empty(777 * n, dtype=torch.bfloat16, device="cuda")
        dist.all_gather_into_tensor(full, a)
        checks["all_gather_into_tensor"] = bool(torch.equal(
            full, torch.arange(n, device="cuda").repeat_interleave(777).to(torch.bfloat16)))
        parts = [torch.empty(777, dtype=torch.bfloat16, device="cuda") for _ in range(n)]
        dist.all_gather(parts, a)
        checks["all_gather_list"] = all(bool(torch.all(p == q).item()) for q, p in enumerate(parts))
        # --- broadcast of a 0-dim tensor (a seed or a loss; ADVICE r02: the byte view needs a reshape first)
        seed = torch.tensor(1000.0 + rank, device="cuda")
        dist.broadcast(seed, src=n - 1)
        checks["broadcast_0dim"] = float(seed.item()) == 1000.0 + (n - 1)
        # --- work.wait(timeout) blocks until the collective is done and reports success
        wz = torch.full((4096,), 2.0, device="cuda")
        work = dist.all_reduce(wz, async_op=True)
        work.wait(timeout=datetime.timedelta(seconds=60))
        checks["wait_timeout_and_success"] = work.is_success() and bool(torch.all(wz == 2.0 * n).item())
        # --- async work on a side stream, then wait() orders the current stream after it
        s = torch.cuda.Stream()
        z = torch.full((1 << 20,), 1.0, device="cuda")
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            work = dist.all_reduce(z, async_op=True)
        work.wait()
        checks["async_wait"] = bool(torch.all(z == n).item())
        # --- captured in a HIP graph (after the communicator's first call, its set-up) and replayed twice
        if n > 1:
            gx = torch.zeros(4099, device="cuda")
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                dist.all_reduce(gx)
            replays = []
            for rep in range(2):
                gx.fill_(float(rank + 1 + rep))
                graph.replay()
                torch.cuda.synchronize()
                replays.append(bool(torch.all(gx == sum(r + 1 + rep for r in range(n))).item()))
            checks["graph_replay"] = all(replays)
        # --- unsupported op and dtype surface as errors, not wrong data
        try:
            dist.all_reduce(torch.ones(4, device="cuda"), op=dist.ReduceOp.AVG)
            checks["avg_refused"] = False
        except ValueError:
            checks["avg_refused"] = True
        dist.barrier()
        dist.destroy_process_group()  # ProcessGroupHCCL.shutdown -> HcclCommDestroy
        progress.write(f"checks {checks}\n")
        q.put((rank, "ok", checks))
    except Exception:  # noqa: BLE001
        progress.write(traceback.format_exc())
        q.put((rank, traceback.format_exc(), None))
        time.sleep(10)


@pytest.mark.parametrize("n,transport", [(1, ""), (2, "ipc"), (4, "ipc")])
def test_reference_pytorch_sample(n, transport):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, n, port, transport, q)) for r in range(n)]
    for p in procs:
        p.start()
    try:
        got = {}
        for _ in procs:
            rank, msg, res = q.get(timeout=240)
            got[rank] = (msg, res)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(n):
        msg, res = got[r]
        assert msg == "ok", f"rank {r}: {msg}"
        assert all(res.values()), f"rank {r}: {res}"


def _ddp_main(rank, n, port, q):
    os.environ["HCCL_AMD_IPC_TIMEOUT_MS"] = "20000"
    os.environ["HCCL_AMD_PG_TRANSPORT"] = "ipc"
    os.makedirs("gpurun_out", exist_ok=True)
    progress = open(f"gpurun_out/process_group_ddp_r{rank}.log", "w", buffering=1)
    try:
        import torch
        import torch.distributed as dist
        from torch.nn.parallel import DistributedDataParallel as DDP
        import hccl_amd.process_group  # noqa: F401

        torch.cuda.set_device(0)
        dist.init_process_group(backend="hccl", rank=rank, world_size=n, init_method=f"tcp://127.0.0.1:{port}",
                                timeout=datetime.timedelta(seconds=120))

        def make(seed):
            torch.manual_seed(seed)
            return torch.nn.Sequential(torch.nn.Linear(512, 256), torch.nn.ReLU(), torch.nn.Linear(256, 8)).cuda()

        checks = {}
        model = make(1000 + rank)  # different on every rank: DDP's start-up broadcast must make them rank 0's
        ddp = DDP(model, device_ids=[0], bucket_cap_mb=1)  # several gradient buckets
        ref = make(1000)
        checks["broadcast_bits"] = all(torch.equal(a, b) for a, b in zip(ddp.module.parameters(), ref.parameters()))
        opt = torch.optim.SGD(ddp.parameters(), lr=0.1)
        ref_opt = torch.optim.SGD(ref.parameters(), lr=0.1)
        for step in range(3):
            xs = [torch.randn(64, 512, generator=torch.Generator().manual_seed(50 * step + r)).cuda() for r in range(n)]
            opt.zero_grad()
            ddp(xs[rank]).square().mean().backward()
            # reference: the mean of every rank's local gradient, on an undistributed copy of the model
            ref_opt.zero_grad()
            for r in range(n):
                (ref(xs[r]).square().mean() / n).backward()
            checks[f"grads_close_{step}"] = all(
                torch.allclose(a.grad, b.grad, rtol=1e-4, atol=1e-6) for a, b in zip(ddp.parameters(), ref.parameters()))
            opt.step()
            ref_opt.step()
        # every rank holds the same parameters, bit for bit, after the steps
        flat = torch.cat([p.detach().reshape(-1) for p in ddp.parameters()])
        everyone = torch.empty(n * flat.numel(), device="cuda")
        dist.all_gather_into_tensor(everyone, flat)
        checks["params_identical"] = all(torch.equal(everyone[r * flat.numel():(r + 1) * flat.numel()], flat)
                                         for r in range(n))
        dist.barrier()
        dist.destroy_process_group()
        progress.write(f"checks {checks}\n")
        q.put((rank, "ok", checks))
    except Exception:  # noqa: BLE001
        progress.write(traceback.format_exc())
        q.put((rank, traceback.format_exc(), None))
        time.sleep(10)


def test_ddp_training_steps_over_the_backend():
    """DistributedDataParallel on the "hccl" backend (2 processes sharing the GPU, IPC communicator): its start-up
    broadcast makes every replica rank 0's bit for bit, three SGD steps average the gradients through HcclAllReduce on
    the backend's CUDA-aware futures (several buckets), and the replicas stay identical."""
    n = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_main, args=(r, n, port, q)) for r in range(n)]
    for p in procs:
        p.start()
    try:
        got = {}
        for _ in procs:
            rank, msg, res = q.get(timeout=240)
            got[rank] = (msg, res)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(n):
        msg, res = got[r]
        assert msg == "ok", f"rank {r}: {msg}"
        assert all(res.values()), f"rank {r}: {res}"
