"""Driver for tools/stream_count_probe.hip: HBM throughput against the number of concurrent streams (NS pure reads,
and NS reads + 1 write: the n-ary fold's shape), over random placements drawn from a pool of 1 GiB buffers, every
shape run on the same placement, interleaved. One JSON line per (kind, NS, U, blocks per CU).
  python tools/stream_count_probe.py > gpurun_out/stream_count.jsonl
"""
import ctypes
import json
import os
import random
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libstream_count_probe.so")
if not os.path.exists(SO):
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC",
                    os.path.join(HERE, "stream_count_probe.hip"), "-o", SO], check=True)
lib = ctypes.CDLL(SO)
lib.probe_streams.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]

GIB = 1 << 30
NS = [int(x) for x in os.environ.get("SC_NS", "1,2,3,4,8").split(",")]
SHAPES = [tuple(int(v) for v in x.split("x")) for x in os.environ.get("SC_SHAPES", "2x1,2x4,1x4").split(",")]
TRIALS = int(os.environ.get("SC_TRIALS", "8"))
POOL = int(os.environ.get("SC_POOL", "12"))


def main():
    torch.cuda.set_device(0)
    pool = [torch.empty(GIB // 4, dtype=torch.float32, device="cuda").uniform_() for _ in range(POOL)]
    sink = torch.empty(256 * 8 * 256 * 4, device="cuda")
    s = torch.cuda.current_stream()
    nvec = GIB // 16
    rng = random.Random(11)
    res = {}
    for _ in range(TRIALS):
        pick = rng.sample(range(POOL), max(NS) + 1)
        cases = [(w, ns, u, bpc) for w in (0, 1) for ns in NS for (bpc, u) in SHAPES]
        rng.shuffle(cases)
        for w, ns, u, bpc in cases:
            ins = (ctypes.c_void_p * 16)(*[pool[i].data_ptr() for i in pick[:ns]])
            out = pool[pick[-1]].data_ptr()
            args = (ns, w, u, bpc, ins, out, sink.data_ptr(), nvec, s.cuda_stream)
            assert lib.probe_streams(*args) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(4):
                lib.probe_streams(*args)
            e1.record(s)
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / 1e3 / 4
            res.setdefault((w, ns, u, bpc), []).append((ns + w) * GIB / t / 1e9)
    for (w, ns, u, bpc), xs in sorted(res.items()):
        xs.sort()
        print(json.dumps({"kind": "read+write" if w else "read", "streams_read": ns, "unroll": u,
                          "blocks_per_cu": bpc, "median_GBps": round(xs[len(xs) // 2], 1),
                          "min_GBps": round(xs[0], 1), "max_GBps": round(xs[-1], 1)}), flush=True)


if __name__ == "__main__":
    main()
