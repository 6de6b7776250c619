"""Soak of the RCCL path: an 8-rank ring AllReduce program (rank 0's, its peers mapped onto a one-rank RCCL
communicator's self loop: tests/test_gpu_rccl.py self_looped) run through HcclAmdCommExecute many thousand times,
eager in the two-stream executor mode (events from the pool, derived waits, RCCL groups on the link stream) and from
a HIP graph, the output compared with the first run's bits every 500 runs.
  python tools/rccl_soak.py > gpurun_out/rccl_soak.jsonl
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import hccl_amd as H  # noqa: E402
from tests.test_gpu_rccl import self_looped  # noqa: E402

RUNS = int(os.environ.get("SOAK_RUNS", "5000"))


def main():
    torch.cuda.set_device(0)
    comm = H.comm_init_root_info(1, H.get_root_info(), 0)
    count = 7 * 8 * 64 * 512  # the ring's 7 rings split evenly: every group pairs up over the self loop
    arr, nops, _ = self_looped(H.OpType.ALLREDUCE, int(H.Algo.RING), 8, 0, count, H.HcclDataType.FP32)
    x = torch.rand(count, device="cuda")
    y = torch.empty_like(x)
    s = torch.cuda.Stream()
    comm.execute(arr, nops, x, y, H.HcclReduceOp.SUM, False, s)
    torch.cuda.synchronize()
    ref = y.clone()
    res = {"program_records": nops, "count": count}
    for mode in ("eager", "graph"):
        bad = 0
        g = None
        if mode == "graph":
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                comm.execute(arr, nops, x, y, H.HcclReduceOp.SUM, False, torch.cuda.current_stream())
        t0 = time.perf_counter()
        for k in range(RUNS):
            if mode == "eager":
                comm.execute(arr, nops, x, y, H.HcclReduceOp.SUM, False, s)
            else:
                g.replay()
            if k % 500 == 499:
                torch.cuda.synchronize()
                bad += 0 if torch.equal(y, ref) else 1
                y.zero_()
                print(f"{mode} {k + 1} runs, {bad} bad, {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
        torch.cuda.synchronize()
        res[mode] = {"runs": RUNS, "bad_checks": bad, "checks": RUNS // 500,
                     "us_per_run": round((time.perf_counter() - t0) / RUNS * 1e6, 1)}
        del g  # a graph holding RCCL work must go before the communicator (HcclCommDestroy waited on it otherwise)
    print(json.dumps(res), flush=True)
    comm.destroy()


if __name__ == "__main__":
    main()
