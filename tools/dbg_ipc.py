import sys, numpy as np, torch
sys.path.insert(0, "/root/repo")
import hccl_amd as H
from oracle import oracle as O
from tests import sched_ref as R
from tests.test_gpu_collectives import collective
n, count = 8, (9 << 20) // 4 + 3
xs = [O.random_operands(O.FP32, count, seed=520 + r, edge=False) for r in range(n)]
want = R.expected(0, 2, O.FP32, O.SUM, xs, count)
for algo in (7, 9, 2, 0):
    comms = H.loopback_world(n)
    used, outs = collective(comms, 0, algo, O.FP32, O.SUM, xs, count)
    bad = np.nonzero(outs[0].view(np.uint32) != want[0].view(np.uint32))[0]
    print(algo, used, "mismatches", len(bad), bad[:10], bad[-5:] if len(bad) else "", flush=True)
    torch.cuda.synchronize()
    for c in comms: c.destroy()
