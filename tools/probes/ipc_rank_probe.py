"""Rank-mode exactness of the one-sided two-shot AllReduce by call size (r03 diagnosis): n processes share the GPU over
the IPC-only communicator; int32 inputs make the sum exact. One JSON line per size: mismatching elements, the first
and last bad index, the staging area size, workgroups and barrier status.
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29591 \\
      tools/ipc_rank_probe.py --mib 16,64,128,200,300
"""
import argparse
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import hccl_amd as H  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", default="16,64,128,200,300")
    ap.add_argument("--algo", default="IPC_TWOSHOT")
    ap.add_argument("--blocks", type=int, default=0)
    # r05: the r03 probe's and test's first form had no synchronisation between the inputs made on the current stream
    # and the collective on s; --no-sync replays that form (the r03 rank-mode wrong result)
    ap.add_argument("--no-sync", action="store_true")
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    os.environ.setdefault("HCCL_AMD_IPC_TIMEOUT_MS", "10000")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def all_gather(b):
        out = [None] * world
        dist.all_gather_object(out, b)
        return out

    comm = H.comm_init_host_exchange(world, rank, all_gather)
    comm.set_algo(H.Algo[args.algo])
    if args.blocks:
        comm.set_ipc_blocks(args.blocks)
    s = torch.cuda.Stream()
    for mib in [int(v) for v in args.mib.split(",")]:
        count = (mib << 20) // 4 + 3
        x = torch.arange(count, device="cuda", dtype=torch.int32) % 1000 + rank
        y = torch.full_like(x, -7)
        if not args.no_sync:
            torch.cuda.synchronize()  # x and y are made on the current stream; the collective runs on s
        comm.all_reduce(x, y, H.HcclReduceOp.SUM, s)
        s.synchronize()
        want = (torch.arange(count, device="cuda", dtype=torch.int32) % 1000) * world + world * (world - 1) // 2
        bad = (y != want).nonzero().flatten()
        untouched = int((y == -7).sum())
        row = {"rank": rank, "mib": mib, "algo": H.Algo(comm.last_algo).name, "bad": int(bad.numel()),
               "untouched": untouched, "first_bad": int(bad[0]) if bad.numel() else None,
               "last_bad": int(bad[-1]) if bad.numel() else None, "count": count,
               "staging_mib": os.environ.get("HCCL_AMD_IPC_STAGING_MIB", "default"),
               "status_bit0": comm.ipc_status() & 1, "synchronised_inputs": not args.no_sync}
        print(json.dumps(row), flush=True)
        del x, y, want, bad
    torch.cuda.synchronize()
    dist.barrier()
    comm.destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
