"""Host-side cost of enqueuing one collective (schedule build + executor: events, waits, launches, transport calls),
measured on a loopback world of n ranks on one GPU (one host thread per rank; the link ops are device copies). The
GPU time is reported beside it, so a host cost well below the GPU time means the host runs ahead of the device.
Usage: python tools/probe_host_overhead.py > gpurun_out/host_overhead.jsonl
"""
import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import hccl_amd as H  # noqa: E402

CASES = [  # (label, op, algo, n, bytes per rank)
    ("C5 1 KiB fp16 AR auto", 0, H.Algo.AUTO, 8, 1 << 10),
    ("C5 1 MiB fp16 AR auto", 0, H.Algo.AUTO, 8, 1 << 20),
    ("C5 64 MiB fp16 AR auto", 0, H.Algo.AUTO, 8, 64 << 20),
    ("C3 1 GiB fp32 AR MeshChunk", 0, H.Algo.AUTO, 8, 1 << 30),
    ("C3 1 GiB fp32 AR ring (7 rings)", 0, H.Algo.RING, 8, 1 << 30),
    ("C4 RS 1 GiB bf16 auto", 1, H.Algo.AUTO, 8, 1 << 30),
]


def main():
    torch.cuda.set_device(0)
    comms = H.loopback_world(8)
    for label, op, algo, n, nbytes in CASES:
        dt = torch.float16 if "fp16" in label else (torch.bfloat16 if "bf16" in label else torch.float32)
        count = nbytes // torch.tensor([], dtype=dt).element_size()
        in_count = count * n if op == 1 else count
        sends = [torch.ones(in_count, dtype=dt, device="cuda") for _ in range(n)]
        recvs = [torch.empty(count, dtype=dt, device="cuda") for _ in range(n)]
        streams = [torch.cuda.Stream() for _ in range(n)]
        for c in comms:
            c.set_algo(algo)
        host = [0.0] * n
        iters = 20 if nbytes <= (64 << 20) else 3

        def body(r):
            t = 0.0
            for _ in range(iters):
                t0 = time.perf_counter()
                if op == 0:
                    comms[r].all_reduce(sends[r], recvs[r], H.HcclReduceOp.SUM, streams[r])
                else:
                    comms[r].reduce_scatter(sends[r], recvs[r], H.HcclReduceOp.SUM, streams[r])
                t += time.perf_counter() - t0
            host[r] = t / iters

        torch.cuda.synchronize()
        g0 = time.perf_counter()
        th = [threading.Thread(target=body, args=(r,)) for r in range(n)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - g0) / iters
        print(json.dumps({"case": label, "algo": H.Algo(comms[0].last_algo).name, "n": n, "bytes": nbytes,
                          "host_us_per_call_max_rank": round(max(host) * 1e6, 1),
                          "wall_us_per_call": round(wall * 1e6, 1)}), flush=True)
        del sends, recvs
    for c in comms:
        c.set_algo(H.Algo.AUTO)
    torch.cuda.synchronize()
    for c in comms:
        c.destroy()


if __name__ == "__main__":
    main()
