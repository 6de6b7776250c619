"""Does the n-ary fold slow down when its inputs sit at the same offset modulo a large power of two (HBM channel /
bank aliasing)? Inputs are views into one allocation at stride 1 GiB + k * skew (input k), for several skews.
  python tools/probe_fold_skew.py > gpurun_out/fold_skew.jsonl
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import hccl_amd as H  # noqa: E402

GIB = 1 << 30
N = 8


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
    count = GIB // 4
    big = torch.empty((N + 1) * GIB + (N + 1) * (8 << 20), dtype=torch.uint8, device="cuda")
    big.random_(0, 64)
    if os.environ.get("PROBE_WARM", "0") == "1":  # 2 s of folds first: clocks and power state settle
        w = [big[k * GIB:(k + 1) * GIB].view(torch.float32) for k in range(N + 1)]
        t_end = time.time() + 2.0
        while time.time() < t_end:
            H.local_reduce_n(w[N], w[:N])
            torch.cuda.synchronize()
    for skew in (0, 256, 4096, 65536, 1 << 20, (2 << 20) + 4096, 3 * 4096 + 256):
        offs = [k * (GIB + skew) for k in range(N + 1)]
        views = [big[o:o + GIB].view(torch.float32) for o in offs]
        out, ins = views[N], views[:N]
        ts = sorted(timeit(lambda: H.local_reduce_n(out, ins)) for _ in range(3))
        t = ts[1]
        print(json.dumps({"n": N, "skew_bytes": skew, "us": round(t * 1e6, 1),
                          "GBps": round((N + 1) * GIB / t / 1e9, 1)}), flush=True)
    # separate allocations, as a caller's buffers would be
    sep = [torch.empty(count, dtype=torch.float32, device="cuda").uniform_() for _ in range(N + 1)]
    ts = sorted(timeit(lambda: H.local_reduce_n(sep[N], sep[:N])) for _ in range(3))
    t = ts[1]
    addrs = [hex(x.data_ptr() % (1 << 32)) for x in sep]
    print(json.dumps({"n": N, "skew_bytes": "separate", "us": round(t * 1e6, 1),
                      "GBps": round((N + 1) * GIB / t / 1e9, 1), "low_addr_bits": addrs}), flush=True)


if __name__ == "__main__":
    main()
