"""Drive the IPC kernel in a loopback world (all n ranks as blockIdx.y of one launch on one GPU) for a kernel trace:
  rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ipc -o run -- python tools/profile_ipc_world.py
One process, no launcher. Prints one JSON line per case with the host-timed average per call."""
import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import hccl_amd as H  # noqa: E402

N = 8
CASES = [("AR", 1 << 10), ("AR", 1 << 20), ("AR", 64 << 20), ("AR", 256 << 20), ("RS", 256 << 20),
         ("AG", 32 << 20)]


def main():
    torch.cuda.set_device(0)
    comms = H.loopback_world(N)
    for c in comms:
        c.set_algo(H.Algo.IPC)
    streams = [torch.cuda.Stream() for _ in range(N)]
    for kind, nbytes in CASES:
        count = nbytes // 4
        if kind == "RS":
            sends = [torch.ones(count, device="cuda") for _ in range(N)]
            recvs = [torch.empty(count // N, device="cuda") for _ in range(N)]
        elif kind == "AG":
            sends = [torch.ones(count // N, device="cuda") for _ in range(N)]
            recvs = [torch.empty(count, device="cuda") for _ in range(N)]
        else:
            sends = [torch.ones(count, device="cuda") for _ in range(N)]
            recvs = [torch.empty(count, device="cuda") for _ in range(N)]
        iters = 50 if nbytes <= (1 << 20) else 10

        def body(r):
            for _ in range(iters):
                if kind == "AR":
                    comms[r].all_reduce(sends[r], recvs[r], H.HcclReduceOp.SUM, streams[r])
                elif kind == "RS":
                    comms[r].reduce_scatter(sends[r], recvs[r], H.HcclReduceOp.SUM, streams[r])
                else:
                    comms[r].all_gather(sends[r], recvs[r], streams[r])

        torch.cuda.synchronize()
        t0 = time.perf_counter()
        th = [threading.Thread(target=body, args=(r,)) for r in range(N)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / iters
        ok = bool(torch.all(recvs[0] == (N if kind != "AG" else 1)).item())
        print(json.dumps({"kind": kind, "n": N, "bytes": nbytes, "us_per_call": round(dt * 1e6, 1),
                          "algo": H.Algo(comms[0].last_algo).name, "ok": ok}), flush=True)
        del sends, recvs
    torch.cuda.synchronize()
    for c in comms:
        c.destroy()


if __name__ == "__main__":
    main()
