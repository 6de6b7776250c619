"""Does the relative placement of a fold's operands change its HBM rate? (r04)

The 8-input ordered fold (k_reduceN, 8 x 1 GiB fp32 in, 1 GiB out) reads 0.70-0.72 of 8 TB/s in the bench at its
median but 0.77 in its best launches (profiles/r02_ab_fold_modes.jsonl: min 1569 us vs median 1702 us). Every lane
loads the same element index of all eight operands, so operands whose bases are congruent modulo the DRAM interleave
period hit the same banks with different rows. This probe places the eight operands in one allocation at a stride of
1 GiB + pad, for several pads, and times the fold interleaved over rounds (HIP events on the launch stream).
  timeout -k 10 300 python3 tools/fold_stagger_probe.py > gpurun_out/fold_stagger.jsonl
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import hccl_amd as H  # noqa: E402

N_IN = 8
COUNT = (1 << 30) // 4  # 1 GiB of fp32 per operand
PADS = [0, 256, 4096, 65536 + 256, 1 << 20, (2 << 20) + 4096, (3 << 20) + 128 * 7]
ROUNDS = int(os.environ.get("STAGGER_ROUNDS", "4"))
REPS = 5


def main():
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    out = torch.empty(COUNT, device="cuda")
    big_stride_max = COUNT * 4 + max(PADS)
    arena = torch.empty(N_IN * big_stride_max // 4 + 64, device="cuda")
    arena.uniform_(-1, 1)
    separate = [torch.rand(COUNT, device="cuda") for _ in range(N_IN)]
    ref = None
    res = {}
    layouts = [("separate", None)] + [(f"pad_{p}", p) for p in PADS]
    for rnd in range(ROUNDS):
        for name, pad in layouts:
            if pad is None:
                srcs = separate
            else:
                stride = (COUNT * 4 + pad) // 4
                srcs = [arena[j * stride:j * stride + COUNT] for j in range(N_IN)]
            with torch.cuda.stream(s):
                H.local_reduce_n(out, srcs, stream=s)  # warm
                evs = [torch.cuda.Event(enable_timing=True) for _ in range(REPS + 1)]
                evs[0].record(s)
                for k in range(REPS):
                    H.local_reduce_n(out, srcs, stream=s)
                    evs[k + 1].record(s)
            torch.cuda.synchronize()
            us = [evs[k].elapsed_time(evs[k + 1]) * 1e3 for k in range(REPS)]
            res.setdefault(name, []).extend(us)
            if name == "pad_0" and rnd == 0:
                ref = torch.stack(srcs).sum(0)  # not bitwise (order), a sanity check only
                ok = torch.allclose(out, ref, atol=1e-4)
                print(json.dumps({"sanity_allclose": bool(ok)}), flush=True)
        print(json.dumps({"round": rnd}), flush=True)
    algo = (N_IN + 1) * COUNT * 4
    for name, v in res.items():
        v = sorted(v)
        med = v[len(v) // 2]
        print(json.dumps({"layout": name, "median_us": round(med, 1), "min_us": round(v[0], 1),
                          "max_us": round(v[-1], 1), "median_TBps": round(algo / med / 1e6, 3),
                          "frac": round(algo / med / 1e6 / 8.0, 4)}), flush=True)


if __name__ == "__main__":
    main()
