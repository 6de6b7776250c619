"""Per-call time of small AllReduces (C5's latency end, fp16) on a loopback world of n ranks on one GPU (one host thread
per rank), with the small-call rule on (HCCL_AMD_SMALL_IPC_BYTES, the default: one launch of the one-sided kernel) and
off (the schedule over the loopback transport), for the auto family and RHD. Every rank issues K calls back to back on
its own stream; per call = wall time of the K calls after a device synchronisation / K. A loopback world meets on the
host for every call (the one-sided kernel's launch is issued by rank 0 after a host all-gather), so these are upper
bounds dominated by the harness, not xGMI numbers; the rank-mode figures are tools/graph_latency.py's.
  python tools/small_call_latency.py > gpurun_out/small_call_latency.jsonl
"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import hccl_amd as H  # noqa: E402

K = int(os.environ.get("PROBE_ITERS", "200"))


def run(comms, xs, ys, streams, k):
    n = len(comms)

    def body(r):
        for _ in range(k):
            comms[r].all_reduce(xs[r], ys[r], H.HcclReduceOp.SUM, streams[r])

    th = [threading.Thread(target=body, args=(r,)) for r in range(n)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def main():
    torch.cuda.set_device(0)
    for n in (2, 4, 8):
        comms = H.loopback_world(n)
        streams = [torch.cuda.Stream() for _ in range(n)]
        for nbytes in (1 << 10, 1 << 14, 1 << 17, 1 << 20):
            xs = [torch.ones(nbytes // 2, dtype=torch.float16, device="cuda") for _ in range(n)]
            ys = [torch.empty_like(x) for x in xs]
            torch.cuda.synchronize()
            for algo in (H.Algo.AUTO, H.Algo.RHD):
                for rule in (1 << 20, 0):
                    for c in comms:
                        c.set_algo(algo)
                        c.set_config(H.Config.SMALL_IPC_BYTES, rule)
                    run(comms, xs, ys, streams, 10)
                    t = run(comms, xs, ys, streams, K)
                    ok = all(bool(torch.all(y == n).item()) for y in ys)
                    print(json.dumps({"n": n, "bytes": nbytes, "algo": algo.name, "small_call_rule": rule,
                                      "ran": H.Algo(comms[0].last_algo).name, "us_per_call": round(t / K * 1e6, 2),
                                      "ok": ok}), flush=True)
        torch.cuda.synchronize()
        for c in comms:
            c.destroy()


if __name__ == "__main__":
    main()
