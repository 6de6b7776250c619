"""Is the 8-input fold's box-to-box spread address translation? (r04)

The ordered 8-input fold (k_reduceN, 8 x 1 GiB fp32 in, 1 GiB out) reads 0.70 of 8 TB/s on most boxes and 0.78-0.79 on
some, and r04's placement probes disagreed between boxes (profiles/r04_fold_stagger_probe.jsonl: one allocation 0.78
against eight separate 0.705; profiles/r04_layout_probe.jsonl: both 0.69). One candidate the byte counters cannot see
is the UTCL1/UTCL2 translation path: nine streams with a front of several MiB each. This probe runs the fold over two
operand sets made in the order --first names (one arena holding all nine buffers, or nine separate allocations), each
timed interleaved (HIP events on the launch stream), and prints the launch order so that a rocprofv3 --pmc pass of the
same command attributes its TCP_UTCL1_* counters per set:
  timeout -k 10 120 python3 tools/fold_tlb_probe.py --first arena > gpurun_out/fold_tlb_arena_first.jsonl
  timeout -s KILL 60 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum \
      TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum -d gpurun_out/tlb -o run -- python3 tools/fold_tlb_probe.py
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import hccl_amd as H  # noqa: E402

N_IN = 8
COUNT = (1 << 30) // 4


def arena_set():
    stride = COUNT + 1024  # 4 KiB apart
    arena = torch.empty((N_IN + 1) * stride, device="cuda")
    arena.uniform_(-1, 1)
    views = [arena[j * stride:j * stride + COUNT] for j in range(N_IN + 1)]
    return views[:N_IN], views[N_IN], arena


def separate_set():
    srcs = [torch.empty(COUNT, device="cuda").uniform_(-1, 1) for _ in range(N_IN)]
    out = torch.empty(COUNT, device="cuda")
    return srcs, out, srcs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--first", choices=("arena", "separate"), default="arena")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=4)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    order = [a.first, "separate" if a.first == "arena" else "arena"]
    sets = {}
    for name in order:
        sets[name] = arena_set() if name == "arena" else separate_set()
    torch.cuda.synchronize()
    res = {name: [] for name in order}
    launch = 0
    for rnd in range(a.rounds):
        for name in order:
            srcs, out, _ = sets[name]
            with torch.cuda.stream(s):
                evs = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps + 1)]
                evs[0].record(s)
                for k in range(a.reps):
                    H.local_reduce_n(out, srcs, stream=s)
                    evs[k + 1].record(s)
            torch.cuda.synchronize()
            res[name].extend(evs[k].elapsed_time(evs[k + 1]) * 1e3 for k in range(a.reps))
            print(json.dumps({"round": rnd, "set": name, "fold_launches": [launch, launch + a.reps - 1]}), flush=True)
            launch += a.reps
    algo = (N_IN + 1) * COUNT * 4
    for name, v in res.items():
        v = sorted(v)
        med = v[len(v) // 2]
        print(json.dumps({"first": a.first, "set": name, "median_us": round(med, 1), "min_us": round(v[0], 1),
                          "max_us": round(v[-1], 1), "frac": round(algo / med / 1e6 / 8.0, 4)}), flush=True)


if __name__ == "__main__":
    main()
