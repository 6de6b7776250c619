"""Soak of the LL form in rank mode (r05): n processes sharing the GPU, 100 calls captured in one HIP graph (AllReduce
and ReduceScatter in turn, each on inputs of its own), replayed SOAK_REPLAYS times. Before every replay the inputs
all grow by one, so a call that read a word of an earlier launch (a flag or parity mix-up) returns a value that differs
from this replay's; every 10th replay every output is checked. Both LL parities are reused SOAK_REPLAYS x 50 times.
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29593 \\
      tools/probes/ll_soak.py > gpurun_out/ll_soak.jsonl
"""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import hccl_amd as H  # noqa: E402

CALLS = 100
ELEMS = 1024  # fp32 per AllReduce call and per ReduceScatter block: 4 KiB, well inside the LL limit
REPLAYS = int(os.environ.get("SOAK_REPLAYS", "10000"))


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    os.environ.setdefault("HCCL_AMD_IPC_TIMEOUT_MS", "20000")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def all_gather(b):
        out = [None] * world
        dist.all_gather_object(out, b)
        return out

    comm = H.comm_init_host_exchange(world, rank, all_gather)
    comm.set_algo(H.Algo.IPC)
    s = torch.cuda.Stream()
    # call k reads row k of X (AllReduce) or of XR (ReduceScatter, n blocks); value rank + 1 + k (+ replays so far)
    k_col = torch.arange(CALLS, device="cuda", dtype=torch.float32).unsqueeze(1)
    X = (k_col + rank + 1).repeat(1, ELEMS).contiguous()
    XR = (k_col + rank + 1).repeat(1, world * ELEMS).contiguous()
    Y = torch.zeros(CALLS, ELEMS, device="cuda")
    comm.all_reduce(X[0], Y[0], H.HcclReduceOp.SUM, s)  # IPC set-up, uncaptured
    torch.cuda.synchronize()
    ll0 = comm.ipc_ll_launches()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=torch.cuda.Stream()):
        cs = torch.cuda.current_stream()
        for k in range(CALLS):
            if k % 2 == 0:
                comm.all_reduce(X[k], Y[k], H.HcclReduceOp.SUM, cs)
            else:
                comm.reduce_scatter(XR[k], Y[k], H.HcclReduceOp.SUM, cs)
    tot_rank = world * (world + 1) / 2
    bad = 0
    checks = 0
    t0 = time.perf_counter()
    for rep in range(REPLAYS):
        X.add_(1)
        XR.add_(1)
        g.replay()
        if rep % 10 == 9:
            torch.cuda.synchronize()
            want = (k_col.squeeze(1) * world + tot_rank + world * (rep + 1)).unsqueeze(1)
            checks += 1
            if not bool(torch.all(Y == want).item()) or comm.ipc_status() & 1:
                bad += 1
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ll = comm.ipc_ll_launches() - ll0
    status = comm.ipc_status()
    dist.barrier()
    if rank == 0:
        calls = REPLAYS * CALLS
        print(json.dumps({"n": world, "calls": calls, "ll_launches": ll, "bad_checks": bad, "checks": checks,
                          "status_bit0": status & 1, "wall_s": round(wall, 1),
                          "us_per_call": round(wall / calls * 1e6, 2)}), flush=True)
    comm.destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
