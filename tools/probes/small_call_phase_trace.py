"""Where a small one-sided AllReduce spends its device time (r05): rank mode, n processes on the one GPU, the kernel's
phase stamps (HCCL_AMD_IPC_TRACE) of the last of K back-to-back eager calls. All processes stamp the same device's
100 MHz clock, so the ranks' rows line up: each rank's kernel entry, its push (phase 0), its barrier wait, its fold and
its exit, and the skew between the ranks' entries.
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 \\
      tools/probes/small_call_phase_trace.py > gpurun_out/small_call_phase_trace.jsonl
"""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import hccl_amd as H  # noqa: E402

K = 200
TR_ENTRY, TR_PHASE0, TR_BARRIER1, TR_PHASE1, TR_EXIT = 0, 2, 3, 4, 7


def main():
    os.environ["HCCL_AMD_IPC_TRACE"] = "1"
    os.environ.setdefault("HCCL_AMD_IPC_TIMEOUT_MS", "10000")
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def all_gather(b):
        out = [None] * world
        dist.all_gather_object(out, b)
        return out

    comm = H.comm_init_host_exchange(world, rank, all_gather)
    comm.set_algo(H.Algo.IPC)
    s = torch.cuda.Stream()
    for nbytes in (1024, 65536, 1 << 20):
        x = torch.ones(nbytes // 4, device="cuda")
        y = torch.empty_like(x)
        torch.cuda.synchronize()
        for mode in ("back_to_back", "isolated"):
            dist.barrier()
            for _ in range(K if mode == "back_to_back" else 1):
                comm.all_reduce(x, y, H.HcclReduceOp.SUM, s)
            s.synchronize()
            tr, blocks = comm.ipc_trace()
            row = tr[rank, :blocks, :].astype(np.int64)
            mine = {"entry_first": int(row[:, TR_ENTRY].min()), "entry_last": int(row[:, TR_ENTRY].max()),
                    "phase0_last": int(row[:, TR_PHASE0].max()), "barrier1_last": int(row[:, TR_BARRIER1].max()),
                    "phase1_last": int(row[:, TR_PHASE1].max()), "exit_last": int(row[:, TR_EXIT].max()),
                    "blocks": blocks}
            rows = all_gather(mine)
            if rank == 0:
                t0 = min(r["entry_first"] for r in rows)
                us = lambda t: round((t - t0) / 100.0, 2)  # noqa: E731  (ticks of 10 ns)
                print(json.dumps({
                    "bytes": nbytes, "mode": mode, "n": world, "ok": bool(torch.all(y == world).item()),
                    "light_fence": os.environ.get("HCCL_AMD_IPC_LIGHT_FENCE", "default (system scope in rank mode)"),
                    "per_rank_us_from_first_entry": [
                        {"entry_first": us(r["entry_first"]), "entry_last": us(r["entry_last"]),
                         "push_done": us(r["phase0_last"]), "barrier_passed": us(r["barrier1_last"]),
                         "fold_done": us(r["phase1_last"]), "exit": us(r["exit_last"]), "blocks": r["blocks"]}
                        for r in rows]}), flush=True)
    dist.barrier()
    comm.destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
