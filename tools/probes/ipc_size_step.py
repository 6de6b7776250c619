"""Is there a step in the one-sided kernel's time between 128 and 256 MiB? (the r01 one-GPU harness
line read 261.8 us at 128 MiB and 1028.9 us at 256 MiB for the IPC row, while the rows before it, which ran the same
path, read 250.7 and 472.9 us.)

n ranks as separate processes sharing the one GPU (IPC-only communicators, as tests/test_gpu_ipc_ranks.py), fp16 SUM
AllReduce, sizes interleaved over several rounds so that no size is measured in one burst; per size the median, min
and max over rounds of the per-call time (max over ranks), for the auto family (IPC) and the fixed two-shot
(IPC_TWOSHOT). Not an xGMI measurement: both ranks share one GPU's HBM.
  python tools/ipc_size_step.py > gpurun_out/ipc_size_step.jsonl
"""
import datetime
import json
import multiprocessing as mp
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SIZES = [int(x) << 20 for x in os.environ.get("STEP_MIB", "32,64,128,192,256,384,512").split(",")]
ROUNDS = int(os.environ.get("STEP_ROUNDS", "5"))
ITERS = int(os.environ.get("STEP_ITERS", "5"))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, n, port, q):
    sys.path.insert(0, ROOT)
    os.environ["HCCL_AMD_IPC_TIMEOUT_MS"] = "20000"
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=n,
                            timeout=datetime.timedelta(seconds=300))
    torch.cuda.set_device(0)
    import hccl_amd as H

    def all_gather(b):
        out = [None] * n
        dist.all_gather_object(out, b)
        return out

    comm = H.comm_init_host_exchange(n, rank, all_gather)
    s = torch.cuda.Stream()
    big = max(SIZES)
    x = torch.rand(big // 2, device="cuda").half()
    y = torch.empty_like(x)
    res = {}
    for rnd in range(ROUNDS):
        order = SIZES[rnd % len(SIZES):] + SIZES[:rnd % len(SIZES)]  # rotate the start size every round
        for nbytes in order:
            for algo in (H.Algo.IPC, H.Algo.IPC_TWOSHOT):
                comm.set_algo(algo)
                a, b = x[: nbytes // 2], y[: nbytes // 2]
                comm.all_reduce(a, b, H.HcclReduceOp.SUM, s)
                s.synchronize()
                dist.barrier()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(ITERS):
                    comm.all_reduce(a, b, H.HcclReduceOp.SUM, s)
                e1.record(s)
                s.synchronize()
                t = e0.elapsed_time(e1) * 1e3 / ITERS
                tmax = max(all_gather(t))
                res.setdefault((algo.name, nbytes), []).append(tmax)
    status = comm.ipc_status()
    dist.barrier()
    comm.destroy()
    dist.destroy_process_group()
    q.put((rank, res, status))


def main():
    n = int(os.environ.get("STEP_RANKS", "2"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, n, port, q)) for r in range(n)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        r, res, status = q.get(timeout=600)
        got[r] = (res, status)
    for p in procs:
        p.join(timeout=60)
    res, status = got[0]
    for (algo, nbytes), ts in sorted(res.items(), key=lambda kv: (kv[0][0], kv[0][1])):
        ts = sorted(ts)
        print(json.dumps({"ranks": n, "algo": algo, "bytes": nbytes, "median_us": round(ts[len(ts) // 2], 1),
                          "min_us": round(ts[0], 1), "max_us": round(ts[-1], 1), "rounds": len(ts),
                          "barrier_timeouts": status & 1}), flush=True)
    time.sleep(1)


if __name__ == "__main__":
    main()
