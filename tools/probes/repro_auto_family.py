"""Repeats test_gpu_collectives.py::test_ipc_follows_auto_family[0-4-4099-None] in one process (r03 diagnosis): on a
4-rank loopback world, the one-sided one-shot AllReduce (HCCL_AMD_ALGO_IPC) then the auto (executor, loopback
transport) AllReduce on the same inputs, both compared with the closed form O1 of every rank. Alternates the
barrier fences per call. One JSON line per iteration that mismatches, and a summary.
  timeout -k 10 200 python3 tools/repro_auto_family.py > gpurun_out/repro_auto_family.jsonl
"""
import json
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import hccl_amd as H  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests import sched_ref as R  # noqa: E402
from tests._util import to_device, to_host  # noqa: E402

ITERS = int(os.environ.get("REPRO_ITERS", "30"))


def run(comms, algo, xs, count):
    n = len(comms)
    sends = [to_device(O.FP32, x) for x in xs]
    recvs = [to_device(O.FP32, np.zeros(count, np.float32)) for _ in range(n)]
    streams = [torch.cuda.Stream() for _ in range(n)]
    for c in comms:
        c.set_algo(algo)
    torch.cuda.synchronize()
    th = [threading.Thread(target=lambda r=r: comms[r].all_reduce(sends[r], recvs[r], H.HcclReduceOp.SUM, streams[r]))
          for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    ins_after = [to_host(O.FP32, s) for s in sends]
    return [to_host(O.FP32, r) for r in recvs], ins_after


def main():
    torch.cuda.set_device(0)
    n, count = 4, 4099
    comms = H.loopback_world(n)
    xs = [O.random_operands(O.FP32, count, seed=520 + r, edge=False) for r in range(n)]
    family = H.select_algo(0, n, count * 4, False)
    want = R.expected(0, family, O.FP32, O.SUM, xs, count)
    bad_total = {"ipc": 0, "auto": 0, "inputs": 0}
    for it in range(ITERS):
        os.environ["HCCL_AMD_IPC_LIGHT_FENCE"] = str(it % 2 ^ 1)
        row = {"iter": it, "light_fence": it % 2 ^ 1}
        for name, algo in (("ipc", 9), ("auto", 0)):
            outs, ins_after = run(comms, algo, xs, count)
            bad = [int(np.count_nonzero(outs[r].view(np.uint32) != want[r].view(np.uint32))) for r in range(n)]
            moved = [int(np.count_nonzero(ins_after[r].view(np.uint32) != xs[r].view(np.uint32))) for r in range(n)]
            row[name] = bad
            row[name + "_inputs_changed"] = moved
            bad_total[name] += sum(1 for b in bad if b)
            bad_total["inputs"] += sum(1 for m in moved if m)
        if any(row["ipc"]) or any(row["auto"]) or any(row["ipc_inputs_changed"]) or any(row["auto_inputs_changed"]):
            print(json.dumps(row), flush=True)
    print(json.dumps({"summary": bad_total, "iters": ITERS, "family": family, "status": comms[0].ipc_status()}),
          flush=True)
    for c in comms:
        c.destroy()


if __name__ == "__main__":
    main()
