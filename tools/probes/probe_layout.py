"""Does the relative placement of the C2 operands matter? (HBM channel/bank mapping of two streams whose addresses
differ only in high bits.) The fp32 SUM local reduce (default launch) over 2 x 1 GiB, with dst placed at
src + 1 GiB + skew inside one allocation, for several skews, against two separate allocations; interleaved rounds.
Prints one JSON line per layout: median / min / max GB/s of algorithmic bytes (3 GiB per launch)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import hccl_amd as H  # noqa: E402

N = 1 << 28
ROUNDS = 5
REPS = 10
SKEWS_B = [0, 256, 4096, 64 << 10, (2 << 20) + 4096, (1 << 20) * 3 + 1024 * 5, 96 << 20]


def main():
    torch.cuda.set_device(0)
    big = torch.empty(2 * N + max(SKEWS_B) // 4 + 1024, device="cuda")
    big.uniform_(-1, 1)
    sep_src = torch.rand(N, device="cuda") * 2 - 1
    sep_dst = torch.rand(N, device="cuda") * 2 - 1
    layouts = {"separate": (sep_src, sep_dst)}
    for sk in SKEWS_B:
        layouts[f"skew_{sk}"] = (big[:N], big[N + sk // 4: 2 * N + sk // 4])
    res = {k: [] for k in layouts}
    s = torch.cuda.current_stream()
    for _ in range(ROUNDS):
        for k, (src, dst) in layouts.items():
            H.local_reduce(dst, src)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(REPS):
                H.local_reduce(dst, src)
            e1.record(s)
            torch.cuda.synchronize()
            res[k].append(3 * N * 4 / (e0.elapsed_time(e1) / 1e3 / REPS))
    for k, xs in res.items():
        xs.sort()
        print(json.dumps({"layout": k, "dst_minus_src_B": int(layouts[k][1].data_ptr() - layouts[k][0].data_ptr()),
                          "median_GBps": round(xs[len(xs) // 2] / 1e9, 1), "min_GBps": round(xs[0] / 1e9, 1),
                          "max_GBps": round(xs[-1] / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
