"""Ordered n-ary fold (k_reduceN, the mesh schedules' reduce) per dtype at n = 2, 4, 8: 1 GiB per input so the
working set stays far above the 256 MiB Infinity Cache. Algorithmic bytes = (n + 1) x input bytes.
  python tools/sweep_fold_dtypes.py > gpurun_out/fold_dtypes.jsonl
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import hccl_amd as H  # noqa: E402

GIB = 1 << 30


def timeit(fn, reps):
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
    raw = [torch.empty(GIB, dtype=torch.uint8, device="cuda").random_(0, 64) for _ in range(9)]
    for dt in (torch.bfloat16, torch.float16, torch.float32, torch.int8):
        bufs = [r.view(dt) for r in raw]
        for n in (2, 4, 8):
            out = bufs[8]
            ts = sorted(timeit(lambda: H.local_reduce_n(out, bufs[:n]), 5) for _ in range(3))
            t = ts[1]
            nbytes = (n + 1) * GIB
            print(json.dumps({"dtype": str(dt), "n": n, "us": round(t * 1e6, 1), "GBps": round(nbytes / t / 1e9, 1),
                              "frac_8TBps": round(nbytes / t / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
