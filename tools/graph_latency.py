"""Per-call latency of the IPC AllReduce, eager vs captured in a HIP graph (K calls per graph, one replay), in rank
mode on the one-GPU box (n processes share the GPU over the IPC-only communicator; not an xGMI measurement).
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 \\
      tools/graph_latency.py [--algo IPC|IPC_RHD|IPC_TWOSHOT] > gpurun_out/graph_latency.jsonl
"""
import argparse
import json
import os
import sys

import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hccl_amd as H  # noqa: E402

K = 100
T0 = time.time()


def progress(rank, what):
    print(f"[graph_latency] rank {rank} +{time.time() - T0:.1f}s {what}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--algo", default="IPC")
    ap.add_argument("--sizes", default="1024,65536,1048576")
    ap.add_argument("--op", default="ar", choices=["ar", "rs"], help="AllReduce, or ReduceScatter (size = input)")
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    os.environ.setdefault("HCCL_AMD_IPC_TIMEOUT_MS", "10000")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def all_gather(b):
        out = [None] * world
        dist.all_gather_object(out, b)
        return out

    progress(rank, "process group up")
    comm = H.comm_init_host_exchange(world, rank, all_gather)
    progress(rank, "communicator up")
    comm.set_algo(H.Algo[args.algo])
    s = torch.cuda.Stream()
    for nbytes in [int(v) for v in args.sizes.split(",")]:
        x = torch.ones(nbytes // 2, dtype=torch.float16, device="cuda")
        y = torch.empty_like(x) if args.op == "ar" else torch.empty(nbytes // 2 // world, dtype=torch.float16,
                                                                    device="cuda")

        def call(st):
            if args.op == "ar":
                comm.all_reduce(x, y, H.HcclReduceOp.SUM, st)
            else:
                comm.reduce_scatter(x, y, H.HcclReduceOp.SUM, st)
        torch.cuda.synchronize()  # x is made on the current stream; the collectives run on s
        for i in range(10):
            call(s)
            if i == 0:
                progress(rank, f"{nbytes} B: first call enqueued ({H.Algo(comm.last_algo).name})")
                s.synchronize()
                progress(rank, f"{nbytes} B: first call done, ipc status {comm.ipc_status()}")
        torch.cuda.synchronize()
        progress(rank, f"{nbytes} B: warm")
        dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        H.host_profile(reset=True)
        h0 = time.perf_counter()
        for _ in range(K):
            call(s)
        enqueue = (time.perf_counter() - h0) / K * 1e3  # host ms per call (the calls return before the device work)
        # with HCCL_AMD_HOST_PROFILE=1: the library's own host time per call (the entry past its argument checks, and
        # the one-sided launch within it); the rest of `enqueue` is this script's Python and ctypes
        prof = H.host_profile(reset=True)
        lib_us = {k: round(prof[k][0] / max(1, prof[k][1]) / 1e3, 2) for k in ("entry", "ipc") if prof[k][1]}
        e1.record(s)
        torch.cuda.synchronize()
        eager = e0.elapsed_time(e1) / K
        progress(rank, f"{nbytes} B: eager timed")
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=torch.cuda.Stream()):
            cs = torch.cuda.current_stream()
            for _ in range(K):
                call(cs)
        torch.cuda.synchronize()
        progress(rank, f"{nbytes} B: captured")
        g.replay()
        torch.cuda.synchronize()
        progress(rank, f"{nbytes} B: replayed once")
        dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        cur = torch.cuda.current_stream()
        e0.record(cur)
        for _ in range(5):
            g.replay()
        e1.record(cur)
        torch.cuda.synchronize()
        graph = e0.elapsed_time(e1) / (5 * K)
        ok = bool(torch.all(y == world).item())
        t = torch.tensor([eager, graph, enqueue])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if rank == 0:
            print(json.dumps({"op": args.op, "algo": H.Algo(comm.last_algo).name, "n": world, "bytes": nbytes, "eager_us": round(float(t[0]) * 1e3, 2),
                              "graph_us": round(float(t[1]) * 1e3, 2), "enqueue_us": round(float(t[2]) * 1e3, 2),
                              "library_host_us": lib_us,
                              "ok": ok,
                              "ipc_status_bit0": comm.ipc_status() & 1,
                              "light_fence": os.environ.get("HCCL_AMD_IPC_LIGHT_FENCE", "default")}), flush=True)
        del g
    torch.cuda.synchronize()
    dist.barrier()
    comm.destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
