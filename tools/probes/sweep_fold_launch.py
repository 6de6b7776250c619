"""Launch shape of the ordered n-ary fold (k_reduceN): workgroups per CU x vectors per lane, per n, fp32 SUM, 1 GiB per
input (separate allocations). Rounds are interleaved so clock or placement drift hits every shape alike.
  python tools/sweep_fold_launch.py > gpurun_out/fold_launch.jsonl
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import hccl_amd as H  # noqa: E402

GIB = 1 << 30
SHAPES = [tuple(int(v) for v in x.split("x")) for x in os.environ.get("FOLD_SHAPES", "").split(",") if x] or [
    (1, 1), (2, 1), (4, 1), (8, 1), (1, 2), (2, 2), (4, 2), (1, 4), (2, 4)]
ROUNDS = int(os.environ.get("FOLD_ROUNDS", "3"))
NS = tuple(int(x) for x in os.environ.get("FOLD_NS", "2,4,8").split(","))


def timeit(fn, reps=5):
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
    bufs = [torch.empty(GIB // 4, dtype=torch.float32, device="cuda").uniform_() for _ in range(9)]
    out = bufs[8]
    res = {}
    for _ in range(ROUNDS):
        for n in NS:
            for bpc, u in SHAPES:
                H.set_reduce_launch(bpc, u, 0)
                t = timeit(lambda: H.local_reduce_n(out, bufs[:n]))
                res.setdefault((n, bpc, u), []).append(t)
    H.set_reduce_launch(0, 0, 0)
    for (n, bpc, u), ts in sorted(res.items()):
        t = sorted(ts)[len(ts) // 2]
        print(json.dumps({"n": n, "blocks_per_cu": bpc, "unroll": u, "us": round(t * 1e6, 1), "min_us": round(min(ts) * 1e6, 1), "max_us": round(max(ts) * 1e6, 1),
                          "GBps": round((n + 1) * GIB / t / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
