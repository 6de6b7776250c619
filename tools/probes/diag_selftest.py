"""Exercises tests/_stale_diag.py on the GPU with a planted mismatch (the diagnosis code itself, not a finding):
a 4-rank loopback one-shot AllReduce, then diagnose() against a closed form with element 1024 of rank 1 altered.
  timeout -k 10 120 python3 tools/diag_selftest.py
"""
import os
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import hccl_amd as H  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests import sched_ref as R  # noqa: E402
from tests._stale_diag import diagnose  # noqa: E402
from tests._util import to_device, to_host  # noqa: E402


def main():
    n, count = 4, 4099
    comms = H.loopback_world(n)
    xs = [O.random_operands(O.FP32, count, seed=520 + r, edge=False) for r in range(n)]
    sends = [to_device(O.FP32, x) for x in xs]
    recvs = [torch.zeros(count, device="cuda") for _ in range(n)]
    streams = [torch.cuda.Stream() for _ in range(n)]
    torch.cuda.synchronize()
    th = [threading.Thread(target=lambda r=r: comms[r].all_reduce(sends[r], recvs[r], O.SUM, streams[r]))
          for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    family = comms[0].last_algo
    outs = [to_host(O.FP32, r) for r in recvs]
    want = R.expected(0, family, O.FP32, O.SUM, xs, count)
    assert all(np.array_equal(outs[r].view(np.uint32), want[r].view(np.uint32)) for r in range(n))
    want[1] = want[1].copy()
    want[1][1024] += np.float32(1.0)
    rep = diagnose(comms, 0, family, xs, count, 0, want, outs, sends, recvs)
    print(rep)
    f = rep["folds"][0]
    assert f["rank"] == 1 and f["bad"] == 1 and f["refold_bad"] == 1 and f["refold_after_l2_maintain_bad"] == 1
    assert all(len(o["matches_rank"]) == 1 and sum(o["xcc_first_look"]["plain_bad_by_xcc"]) == 0 for o in f["operands"]), f["operands"]
    for c in comms:
        c.destroy()
    print("diag selftest ok")


if __name__ == "__main__":
    main()
