"""Copy and reduce-shaped streams with the source (or the destination) in uncached memory (hipDeviceMallocUncached,
the IPC staging's type) against the same streams on ordinary device memory. Uses tools/hbm_probe.hip's kernels.
  python tools/probe_uncached.py > gpurun_out/probe_uncached.jsonl
"""
import ctypes
import json
import os
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libhbm_probe.so")
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC",
                os.path.join(HERE, "hbm_probe.hip"), "-o", SO], check=True)
lib = ctypes.CDLL(SO)
lib.probe_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
lib.probe_alloc_uncached.restype = ctypes.c_void_p
lib.probe_alloc_uncached.argtypes = [ctypes.c_uint64]
lib.probe_free.argtypes = [ctypes.c_void_p]
GIB = 1 << 30


def main():
    torch.cuda.set_device(0)
    n = GIB // 4
    a = torch.rand(n, device="cuda")
    b = torch.rand(n, device="cuda")
    o = torch.empty(n, device="cuda")
    sink = torch.empty(256 * 8 * 256 * 4, device="cuda")
    ua = lib.probe_alloc_uncached(GIB)
    uo = lib.probe_alloc_uncached(GIB)
    assert ua and uo
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    nvec = n // 4
    # (label, kind, variant, a, b, o, bytes): kind 2 copy, kind 3 r2w1; variant 0 = U 1, nt loads + nt stores
    cases = [("copy cached->cached", 2, 0, a.data_ptr(), a.data_ptr(), o.data_ptr(), 2 * GIB),
             ("copy uncached->cached", 2, 0, ua, ua, o.data_ptr(), 2 * GIB),
             ("copy cached->uncached", 2, 0, a.data_ptr(), a.data_ptr(), uo, 2 * GIB),
             ("r2w1 cached", 3, 0, a.data_ptr(), b.data_ptr(), o.data_ptr(), 3 * GIB),
             ("r2w1 one input uncached", 3, 0, ua, b.data_ptr(), o.data_ptr(), 3 * GIB)]
    res = {c[0]: [] for c in cases}
    for _ in range(5):
        for label, k, v, pa, pb, po, nbytes in cases:
            args = (k, v, 2, pa, pb, po, nvec, sink.data_ptr(), s.cuda_stream)
            assert lib.probe_launch(*args) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(5):
                lib.probe_launch(*args)
            e1.record(s)
            torch.cuda.synchronize()
            res[label].append(nbytes * 5 / (e0.elapsed_time(e1) / 1e3) / 1e9)
    for label, xs in res.items():
        xs.sort()
        print(json.dumps({"case": label, "median_GBps": round(xs[len(xs) // 2], 1), "max_GBps": round(xs[-1], 1)}))
    torch.cuda.synchronize()
    lib.probe_free(ua)
    lib.probe_free(uo)


if __name__ == "__main__":
    main()
