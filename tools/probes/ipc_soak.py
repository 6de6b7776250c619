"""Soak of the one-sided IPC path in rank mode: a million small AllReduces (HIP-graph replays of 100 captured calls)
on n processes sharing the GPU, the result and the barrier status checked every 1,000 replays. It exercises the
device-side barrier epochs far past anything the tests reach (2 epochs per call, wrap-safe compare: ADVICE r01).
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29591 \\
      tools/ipc_soak.py > gpurun_out/ipc_soak.jsonl
"""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import hccl_amd as H  # noqa: E402

CALLS_PER_GRAPH = 100
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
    comm.set_algo(H.Algo.IPC_TWOSHOT)  # two barriers per call
    s = torch.cuda.Stream()
    x = torch.zeros(256, device="cuda")
    y = torch.zeros(256, device="cuda")
    comm.all_reduce(x, y, H.HcclReduceOp.SUM, s)  # IPC set-up, uncaptured
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=torch.cuda.Stream()):
        cs = torch.cuda.current_stream()
        for _ in range(CALLS_PER_GRAPH):
            comm.all_reduce(x, y, H.HcclReduceOp.SUM, cs)
    bad = 0
    t0 = time.perf_counter()
    for rep in range(REPLAYS):
        if rep % 1000 == 0:
            x.fill_(float(rank + 1 + rep % 7))
        g.replay()
        if rep % 1000 == 999:
            torch.cuda.synchronize()
            want = float(sum(r + 1 + (rep - 999) % 7 for r in range(world)))
            if not bool(torch.all(y == want).item()) or comm.ipc_status() & 1:
                bad += 1
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    status = comm.ipc_status()
    dist.barrier()
    if rank == 0:
        calls = REPLAYS * CALLS_PER_GRAPH
        print(json.dumps({"n": world, "calls": calls, "barrier_epochs_per_block": 2 * calls, "bad_checks": bad,
                          "checks": REPLAYS // 1000, "status_bit0": status & 1, "wall_s": round(wall, 1),
                          "us_per_call": round(wall / calls * 1e6, 2)}), flush=True)
    comm.destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
