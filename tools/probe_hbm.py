"""Driver for tools/hbm_probe.hip: HBM ceilings of read / write / copy / reduce-shaped streams on MI355X,
interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24). Prints one JSON line per variant."""
import ctypes
import json
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libhbm_probe.so")
if not os.path.exists(SO):
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC",
                    os.path.join(HERE, "hbm_probe.hip"), "-o", SO], check=True)
lib = ctypes.CDLL(SO)
lib.probe_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]

GIB = 1 << 30
BYTES = {0: 2 * GIB, 1: GIB, 2: 2 * GIB, 3: 3 * GIB, 4: 3 * GIB, 5: 3 * GIB}
NAMES = {0: "read2", 1: "write1", 2: "copy", 3: "r2w1", 4: "r2w1buf", 5: "r2w1lds"}
VARIANTS = {0: [0, 1, 2, 3], 1: [0, 1, 2, 3], 2: [0, 1, 2, 3], 3: [0, 1, 2],
            4: [0, 1, 2, 3, 4, 5, 6, 7, 8], 5: [0, 1, 2, 3]}


def main():
    torch.cuda.set_device(0)
    n = GIB // 4
    a = torch.rand(n, device="cuda")
    b = torch.rand(n, device="cuda")
    o = torch.empty(n, device="cuda")
    sink = torch.empty(256 * 8 * 256 * 4, device="cuda")
    s = torch.cuda.current_stream()
    nvec = n // 4
    cases = [(k, v, bp) for k, vs in VARIANTS.items() for v in vs for bp in (1, 2, 4)]
    res = {c: [] for c in cases}
    for _ in range(int(os.environ.get("ROUNDS", 4))):
        for c in cases:
            k, v, bp = c
            args = (k, v, bp, a.data_ptr(), b.data_ptr(), o.data_ptr(), nvec, sink.data_ptr(), s.cuda_stream)
            assert lib.probe_launch(*args) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(5):
                lib.probe_launch(*args)
            e1.record(s)
            torch.cuda.synchronize()
            res[c].append(BYTES[k] * 5 / (e0.elapsed_time(e1) / 1e3) / 1e9)
    rows = []
    for (k, v, bp), xs in res.items():
        xs.sort()
        rows.append({"kind": NAMES[k], "variant": v, "blocks_per_cu": bp, "median_GBps": round(xs[len(xs) // 2], 1),
                     "max_GBps": round(xs[-1], 1)})
    rows.sort(key=lambda r: (r["kind"], -r["median_GBps"]))
    for r in rows:
        print(json.dumps(r))
    # correctness of the reduce-shaped variants
    for k, v in [(3, 0), (4, 0), (4, 2), (5, 1)]:
        o.zero_()
        lib.probe_launch(k, v, 2, a.data_ptr(), b.data_ptr(), o.data_ptr(), nvec, sink.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        print(json.dumps({"check": NAMES[k], "variant": v, "ok": bool(torch.equal(o, a + b))}), file=sys.stderr)


if __name__ == "__main__":
    main()
