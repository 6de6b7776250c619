"""Sweep the IPC kernel's workgroups per launch (HcclAmdCommSetIpcBlocks) against the AllReduce size, in rank mode on
the one-GPU box: n processes share the GPU over the IPC-only communicator (HcclAmdCommInitHostExchange). This is not
an xGMI measurement; it shows the launch/barrier cost per block count at small sizes and the HBM-side effect at large
ones. Run as:
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 \
      tools/probes/sweep_ipc_blocks.py > gpurun_out/sweep_ipc_blocks.jsonl
(SWEEP_BLOCKS / SWEEP_SIZES: comma lists overriding the block counts and byte sizes; SWEEP_ALGO: the family, IPC.)
"""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import hccl_amd as H  # noqa: E402

BLOCKS = tuple(int(x) for x in os.environ.get("SWEEP_BLOCKS", "").split(",") if x) or (16, 32, 64, 128, 256)
SIZES = tuple(int(x) for x in os.environ.get("SWEEP_SIZES", "").split(",") if x) or (
    1 << 10, 1 << 16, 1 << 20, 1 << 24, 1 << 28)


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    os.environ.setdefault("HCCL_AMD_IPC_TIMEOUT_MS", "10000")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def all_gather(b):
        out = [None] * world
        dist.all_gather_object(out, b)
        return out

    comm = H.comm_init_host_exchange(world, rank, all_gather)
    comm.set_algo(H.Algo[os.environ.get("SWEEP_ALGO", "IPC")])
    stream = torch.cuda.Stream()  # a null stream is HCCL_E_PTR, as in the reference's entry checks
    dev = torch.device("cuda", 0)
    for size in SIZES:
        count = size // 2
        send = torch.randn(count, device=dev).half()
        recv = torch.empty_like(send)
        torch.cuda.synchronize()
        iters = 200 if size <= (1 << 20) else (50 if size <= (1 << 24) else 10)
        for blocks in BLOCKS:
            comm.set_ipc_blocks(blocks)
            for _ in range(5):
                comm.all_reduce(send, recv, H.HcclReduceOp.SUM, stream)
            torch.cuda.synchronize()
            dist.barrier()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(iters):
                comm.all_reduce(send, recv, H.HcclReduceOp.SUM, stream)
            e1.record(stream)
            torch.cuda.synchronize()
            t = torch.tensor([e0.elapsed_time(e1) / 1e3 / iters])
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            st = comm.ipc_status()
            if rank == 0:
                us = float(t[0]) * 1e6
                print(json.dumps({"n": world, "bytes": size, "blocks": blocks, "us": round(us, 2),
                                  "busbw_GBps": round(size / (us * 1e-6) * 2 * (world - 1) / world / 1e9, 2),
                                  "algo": H.Algo(comm.last_algo).name, "ipc_status": st}), flush=True)
        del send, recv
    comm.set_ipc_blocks(0)
    comm.destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    t0 = time.time()
    main()
