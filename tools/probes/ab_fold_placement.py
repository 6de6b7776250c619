"""A/B of fold launch shapes over many buffer placements: a pool of 1 GiB buffers, and for each trial a random choice
of n inputs + 1 output from it; every shape runs on the same choice, interleaved. Reports per-shape median, min and
max over the trials, so a shape is judged over placements rather than on one lucky or unlucky layout.
  python tools/ab_fold_placement.py > gpurun_out/ab_fold.jsonl
"""
import json
import os
import random
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import hccl_amd as H  # noqa: E402

GIB = 1 << 30
# bpc x unroll [x fold mode [x cache policy]]: HcclAmdSetFoldMode (0 default, 1 serial, 2 prefetch, 3 every operand
# first); HcclAmdSetReduceLaunch's cachePolicy (0 default, 1 plain, 2 nt loads, 3 nt stores, 4 nt loads + stores)
SHAPES = [tuple(int(v) for v in (x + "x0x0x0").split("x")[:4])
          for x in os.environ.get("AB_SHAPES", "2x2,2x4,4x2,2x1").split(",")]
NS = tuple(int(x) for x in os.environ.get("AB_NS", "8").split(","))
TRIALS = int(os.environ.get("AB_TRIALS", "12"))
POOL = int(os.environ.get("AB_POOL", "20"))


def timeit(fn, reps=4):
    s = torch.cuda.current_stream()
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3 / reps


def main():
    torch.cuda.set_device(0)
    pool = [torch.empty(GIB // 4, dtype=torch.float32, device="cuda").uniform_() for _ in range(POOL)]
    rng = random.Random(7)
    res = {}
    mismatch = set()
    for n in NS:
        for _ in range(TRIALS):
            pick = rng.sample(range(POOL), n + 1)
            ins, out = [pool[i] for i in pick[:n]], pool[pick[n]]
            order = SHAPES[:]
            rng.shuffle(order)
            ref = None
            for bpc, u, fm, pol in order:
                H.set_reduce_launch(bpc, u, pol)
                H.set_fold_mode(fm)
                res.setdefault((n, bpc, u, fm, pol), []).append(timeit(lambda: H.local_reduce_n(out, ins)))
                # every shape and mode folds in the same order: the outputs must be identical bits
                digest = out.view(torch.int32)[:: 1 << 10].clone()
                if ref is None:
                    ref = digest
                elif not torch.equal(ref, digest):
                    mismatch.add((n, bpc, u, fm, pol))
    H.set_reduce_launch(0, 0, 0)
    H.set_fold_mode(0)
    for (n, bpc, u, fm, pol), ts in sorted(res.items()):
        ts = sorted(ts)
        med = ts[len(ts) // 2]
        print(json.dumps({"n": n, "blocks_per_cu": bpc, "unroll": u, "fold_mode": fm, "cache_policy": pol,
                          "bits_match": (n, bpc, u, fm, pol) not in mismatch, "median_us": round(med * 1e6, 1),
                          "min_us": round(ts[0] * 1e6, 1), "max_us": round(ts[-1] * 1e6, 1),
                          "mean_us": round(sum(ts) / len(ts) * 1e6, 1),
                          "median_GBps": round((n + 1) * GIB / med / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
