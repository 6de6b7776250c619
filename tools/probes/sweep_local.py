"""Launch-configuration sweep of the fp32 SUM local reduce (C2 shape), interleaved rounds in one process
(cdna_hip_programming.md §5.4 rule 24). Prints one line per variant: median / min GiB/s and HBM fraction."""
import itertools
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import hccl_amd as H  # noqa: E402

N = int(os.environ.get("SWEEP_COUNT", 1 << 28))
ROUNDS = int(os.environ.get("SWEEP_ROUNDS", 5))
REPS = 10


def main():
    torch.cuda.set_device(0)
    src = torch.rand(N, device="cuda") * 2 - 1
    dst = torch.rand(N, device="cuda") * 2 - 1
    out = torch.empty_like(src)
    # cache policy: 1 plain, 2 nt loads, 3 nt stores, 4 nt both, 5 nt both + contiguous per-workgroup tile runs.
    # SWEEP_QUICK=1: the four best launch shapes only.
    if os.environ.get("SWEEP_QUICK") == "1":
        variants = [(b, u, 4, mode) for b, u in ((2, 1), (1, 2), (2, 2), (1, 1)) for mode in ("inplace", "outofplace")]
    else:
        variants = [(b, u, pol, mode) for b, u, pol in itertools.product([1, 2, 3, 4], [1, 2, 4], [1, 2, 3, 4, 5])
                    for mode in ("inplace",)]
        variants += [(b, u, 4, "outofplace") for b, u in itertools.product([1, 2, 3, 4], [1, 2])]
    res = {v: [] for v in variants}
    s = torch.cuda.current_stream()
    for _ in range(ROUNDS):
        for v in variants:
            b, u, nt, mode = v
            H.set_reduce_launch(b, u, nt)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            H.local_reduce(dst, src) if mode == "inplace" else H.local_reduce2(out, src, dst)
            e0.record(s)
            for _ in range(REPS):
                if mode == "inplace":
                    H.local_reduce(dst, src)
                else:
                    H.local_reduce2(out, src, dst)
            e1.record(s)
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / 1e3 / REPS
            res[v].append(3 * N * 4 / t)
    rows = []
    for v, xs in res.items():
        xs.sort()
        med = xs[len(xs) // 2]
        rows.append((med, v, xs[0], xs[-1]))
    rows.sort(reverse=True)
    for med, v, lo, hi in rows:
        print(json.dumps({"blocks_per_cu": v[0], "unroll": v[1], "policy": v[2], "mode": v[3],
                          "median_GBps": round(med / 1e9, 1), "min_GBps": round(lo / 1e9, 1),
                          "max_GBps": round(hi / 1e9, 1), "frac_hbm": round(med / 8e12, 4)}))
    H.set_reduce_launch(0, 0, 0)


if __name__ == "__main__":
    main()
