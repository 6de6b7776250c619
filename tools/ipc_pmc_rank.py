"""One rank of the one-sided kernel's counter run: n processes share the GPU (rank mode, IPC-only
communicators over a gloo host exchange, as tests/test_gpu_ipc_ranks.py), each a separate program so that rank 0 alone
can run under rocprofv3 (counters are device-wide: rank 0's dispatch window covers every rank's kernel, which the
barriers keep concurrent with it). Launched by tools/gpu_call.sh step `ipc_pmc`:
  python tools/ipc_pmc_rank.py --rank R --world 2 --mib 512 --dtype fp32 --algo IPC_TWOSHOT
Rank 0 prints one JSON line: per-call time (HIP events on the launch stream, max over ranks) and the kernel's
algorithmic bytes per launch summed over the ranks (two-shot AllReduce: 2(3n-2)/n bytes per input byte per rank:
phase 0 reads (n-1)/n of the input and stores it to the owners' slots, phase 1 reads the own chunk and n-1 slots and
writes n results, phase 2 copies n-1 results; on one GPU every one of these lands in the same HBM).
"""
import argparse
import datetime
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--mib", type=int, default=512)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--algo", default="IPC_TWOSHOT")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--port", type=int, default=29611)
    a = ap.parse_args()
    os.environ.setdefault("HCCL_AMD_IPC_TIMEOUT_MS", "30000")
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{a.port}", rank=a.rank, world_size=a.world,
                            timeout=datetime.timedelta(seconds=300))
    torch.cuda.set_device(0)
    import hccl_amd as H

    def all_gather(b):
        out = [None] * a.world
        dist.all_gather_object(out, b)
        return out

    comm = H.comm_init_host_exchange(a.world, a.rank, all_gather)
    comm.set_algo(H.Algo[a.algo])
    tdt = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}[a.dtype]
    count = (a.mib << 20) // torch.tensor([], dtype=tdt).element_size()
    x = torch.rand(count, device="cuda").to(tdt)
    y = torch.empty_like(x)
    s = torch.cuda.Stream()
    for _ in range(2):
        comm.all_reduce(x, y, H.HcclReduceOp.SUM, s)
    s.synchronize()
    dist.barrier()
    torch.empty(1, device="cuda").fill_(7.0)  # trace marker: the timed launches follow the FillFunctor kernel
    torch.cuda.synchronize()
    dist.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.iters):
        comm.all_reduce(x, y, H.HcclReduceOp.SUM, s)
    e1.record(s)
    s.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / a.iters
    us_max = max(all_gather(us))
    status = comm.ipc_status()
    dist.barrier()
    comm.destroy()
    dist.destroy_process_group()
    if a.rank == 0:
        n = a.world
        nbytes = count * x.element_size()
        alg = n * 2 * (3 * n - 2) * nbytes // n if a.algo == "IPC_TWOSHOT" else None
        print(json.dumps({"kernel": "k_ipc_collective", "algo": a.algo, "ranks": n, "dtype": a.dtype,
                          "bytes_per_rank": nbytes, "iters": a.iters, "us_per_call_max_over_ranks": round(us_max, 1),
                          "algorithmic_bytes_per_launch_all_ranks": alg,
                          "achieved_TBps": round(alg / us_max / 1e6, 3) if alg else None,
                          "barrier_timeouts": status & 1}), flush=True)


if __name__ == "__main__":
    main()
