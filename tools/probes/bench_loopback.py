"""Executor overhead on one MI355X: an 8-rank loopback world (one thread per rank, links = device copies) runs
AllReduce at sizes 1 KiB .. 64 MiB; per-call host time and device time per schedule. This is not an xGMI number:
it prices the host side (schedule build, dependency tracking, event/stream calls, transport rendezvous) that every
collective pays, i.e. the floor under config C5's small-message latency."""
import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import hccl_amd as H  # noqa: E402


def main():
    n = int(os.environ.get("LB_RANKS", 8))
    torch.cuda.set_device(0)
    comms = H.loopback_world(n)
    max_bytes = 64 << 20
    sends = [torch.rand(max_bytes // 4, device="cuda") for _ in range(n)]
    recvs = [torch.empty_like(s) for s in sends]
    streams = [torch.cuda.Stream() for _ in range(n)]
    torch.cuda.synchronize()
    rows = []
    for algo in (H.Algo.MESH_ONESHOT, H.Algo.MESH_TWOSHOT, H.Algo.RHD, H.Algo.RING):
        for c in comms:
            c.set_algo(algo)
        nbytes = 1 << 10
        while nbytes <= max_bytes:
            iters = 50 if nbytes <= (1 << 20) else 10
            count = nbytes // 4
            host = [0.0] * n

            def body(r):
                a, b, s = sends[r][:count], recvs[r][:count], streams[r]
                comms[r].all_reduce(a, b, H.HcclReduceOp.SUM, s)  # warm
                s.synchronize()
                t0 = time.perf_counter()
                for _ in range(iters):
                    comms[r].all_reduce(a, b, H.HcclReduceOp.SUM, s)
                host[r] = (time.perf_counter() - t0) / iters
                s.synchronize()

            torch.cuda.synchronize()
            t0 = time.perf_counter()
            th = [threading.Thread(target=body, args=(r,)) for r in range(n)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0)
            rows.append({"algo": algo.name, "bytes": nbytes, "host_us_per_call": round(max(host) * 1e6, 1),
                         "wall_ms_total": round(wall * 1e3, 2), "iters": iters})
            nbytes *= 4
    for c in comms:
        c.destroy()
    for r in rows:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
