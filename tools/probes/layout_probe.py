"""Operand placement and the HBM rate of the reduce kernels (r04).

tools/fold_stagger_probe.py found the 8-input fold at 0.705 of 8 TB/s over eight separate 1 GiB allocations and
0.78-0.79 over eight slices of one allocation. This probe separates the two candidate causes for C2 (dst = src + dst,
2 x 1 GiB fp32) and the 8-input fold: separate allocations as allocated; separate allocations with operand j started
j x 4 KiB + j x 256 B into its own (slightly larger) allocation; slices of one allocation 4 KiB apart. Interleaved
rounds, HIP events on the launch stream, medians.
  timeout -k 10 300 python3 tools/layout_probe.py > gpurun_out/layout_probe.jsonl
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import hccl_amd as H  # noqa: E402

GIB = 1 << 30
COUNT = GIB // 4
STAG = 4096 + 256  # bytes of stagger per operand index


def layouts(n):
    """name -> list of n fp32 views of COUNT elements (kept alive by the returned owners)."""
    out = {}
    sep = [torch.rand(COUNT, device="cuda") for _ in range(n)]
    out["separate"] = (sep, sep)
    own = [torch.rand(COUNT + (j * STAG) // 4, device="cuda") for j in range(n)]
    out["separate_staggered"] = ([own[j][(j * STAG) // 4:(j * STAG) // 4 + COUNT] for j in range(n)], own)
    big = torch.rand(n * (COUNT + 1024) + 16, device="cuda")
    out["one_allocation_4KiB_apart"] = ([big[j * (COUNT + 1024):j * (COUNT + 1024) + COUNT] for j in range(n)], big)
    return out


def time_it(fn, s, reps=5):
    with torch.cuda.stream(s):
        fn()
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
        evs[0].record(s)
        for k in range(reps):
            fn()
            evs[k + 1].record(s)
    torch.cuda.synchronize()
    return [evs[k].elapsed_time(evs[k + 1]) * 1e3 for k in range(reps)]


def main():
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    res = {}
    for kind, n in (("c2", 2), ("fold_n8", 8)):
        ls = layouts(n)
        outbuf = torch.empty(COUNT, device="cuda")
        for _ in range(4):
            for name, (views, _owner) in ls.items():
                if kind == "c2":
                    src, dst = views
                    us = time_it(lambda: H.local_reduce(dst, src, stream=s), s)
                    algo = 3 * GIB
                else:
                    us = time_it(lambda: H.local_reduce_n(outbuf, views, stream=s), s)
                    algo = 9 * GIB
                res.setdefault((kind, name, algo), []).extend(us)
        del ls
        torch.cuda.empty_cache()
    for (kind, name, algo), us in res.items():
        us.sort()
        med = us[len(us) // 2]
        print(json.dumps({"kernel": kind, "layout": name, "median_us": round(med, 1), "min_us": round(us[0], 1),
                          "max_us": round(us[-1], 1), "frac": round(algo / med / 1e6 / 8.0, 4)}), flush=True)


if __name__ == "__main__":
    main()
