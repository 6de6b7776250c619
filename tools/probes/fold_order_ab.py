"""n-ary fold tile order A/B (r04): round-robin tiles over the grid (default) against one contiguous run of tiles per
workgroup (HcclAmdSetReduceLaunch cache policy 5), at several workgroups per CU, n = 3, 4, 8 inputs of 1 GiB fp32 (the
output 1 GiB), interleaved rounds, HIP events on the launch stream; every variant's bits against the default's.
  timeout -k 10 400 python3 tools/fold_order_ab.py > gpurun_out/fold_order_ab.jsonl
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import hccl_amd as H  # noqa: E402

COUNT = (1 << 30) // 4
CFGS = [("default", (0, 0, 0)), ("runs_bpc2_u4", (2, 4, 5)), ("runs_bpc1_u4", (1, 4, 5)), ("runs_bpc4_u4", (4, 4, 5)),
        ("runs_bpc2_u2", (2, 2, 5)), ("rr_bpc1_u4", (1, 4, 4)), ("rr_bpc4_u4", (4, 4, 4))]


def main():
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    srcs = [torch.rand(COUNT, device="cuda") for _ in range(8)]
    out = torch.empty(COUNT, device="cuda")
    ref = torch.empty(COUNT, device="cuda")
    res = {}
    for n in (8, 4, 3):
        H.set_reduce_launch(0, 0, 0)
        H.local_reduce_n(ref, srcs[:n], stream=s)
        torch.cuda.synchronize()
        for rnd in range(3):
            for name, cfg in CFGS:
                H.set_reduce_launch(*cfg)
                with torch.cuda.stream(s):
                    H.local_reduce_n(out, srcs[:n], stream=s)
                    evs = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
                    evs[0].record(s)
                    for k in range(5):
                        H.local_reduce_n(out, srcs[:n], stream=s)
                        evs[k + 1].record(s)
                torch.cuda.synchronize()
                same = bool(torch.equal(out.view(torch.int32), ref.view(torch.int32)))
                r = res.setdefault((n, name), {"us": [], "bits": True})
                r["us"].extend(evs[k].elapsed_time(evs[k + 1]) * 1e3 for k in range(5))
                r["bits"] = r["bits"] and same
    H.set_reduce_launch(0, 0, 0)
    for (n, name), r in res.items():
        us = sorted(r["us"])
        med = us[len(us) // 2]
        algo = (n + 1) * COUNT * 4
        print(json.dumps({"n": n, "variant": name, "median_us": round(med, 1), "min_us": round(us[0], 1),
                          "frac": round(algo / med / 1e6 / 8, 4), "bits_match_default": r["bits"]}), flush=True)


if __name__ == "__main__":
    main()
