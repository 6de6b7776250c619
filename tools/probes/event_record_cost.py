"""Device-side cost of a hipEventRecord between back-to-back small kernels on one stream (r05).

The one-sided kernel's eager calls in rank mode take 15 us each on the device against 9 us from a graph, while the
host enqueues a call in 5.5 us (profiles/r05_small_call_latency_rank_mode.jsonl): the host is not the limit. Every
eager entry records the communicator's tail event on the caller's stream (executor.cc EntryScope); a captured call
does not. This probe times K kernels (torch add, 256 floats to 16 Mi floats) back to back on one stream, alone and
with a disable-timing event recorded after each: a default one (torch's), one with hipEventDisableSystemFence and one
with hipEventReleaseToDevice.
  timeout -k 10 120 python3 tools/probes/event_record_cost.py > gpurun_out/event_record_cost.jsonl
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

K = 2000


def per_launch_us(body, s):
    for _ in range(50):
        body()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(K):
        body()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / K * 1e3


def main():
    torch.cuda.set_device(0)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
    hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    s = torch.cuda.Stream()
    ev = torch.cuda.Event()  # hipEventDisableTiming, like the communicator's tail event
    rows = []
    # 256 floats: the host (Python) sets the pace; 4 Mi floats (32 MiB of traffic, about 6 us of HBM time) and 16 Mi
    # floats (about 21 us): the device does, so a difference there is device time
    for n in (256, 4 << 20, 16 << 20):
        x = torch.zeros(n, device="cuda")
        with torch.cuda.stream(s):
            rows.append({"case": "add", "floats": n, "us": per_launch_us(lambda: x.add_(1), s)})

            def add_rec():
                x.add_(1)
                ev.record(s)

            rows.append({"case": "add+event_record", "floats": n, "us": per_launch_us(add_rec, s)})
            for name, flags in (("disable_system_fence", 0x2 | 0x20000000), ("release_to_device", 0x2 | 0x40000000)):
                ev2 = ctypes.c_void_p()
                assert hip.hipEventCreateWithFlags(ctypes.byref(ev2), ctypes.c_uint(flags)) == 0

                def add_rec2(ev2=ev2):
                    x.add_(1)
                    hip.hipEventRecord(ev2, ctypes.c_void_p(s.cuda_stream))

                rows.append({"case": f"add+event_record({name})", "floats": n, "us": per_launch_us(add_rec2, s)})
    for r in rows:
        r["us"] = round(r["us"], 3)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
