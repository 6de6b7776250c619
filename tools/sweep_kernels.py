"""Roofline table of the shipped reduce kernels on one MI355X (default launch configuration):
  1. every dtype x op of k_reduce2 at 1 GiB per operand (3 streams), HBM GB/s and fraction of 8 TB/s;
  2. the ordered n-ary fold k_reduceN at n = 2..16 over 1 GiB per input ((n+1) streams; 1 GiB keeps the working
     set far above the 256 MiB Infinity Cache, whose hits made 256 MiB inputs read box-dependently fast);
  3. the fp32 SUM local reduce from 1 KiB to 1 GiB per operand (launch latency to bandwidth).
Median of interleaved rounds; algorithmic bytes only. One JSON line per measurement."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hccl_amd as H  # noqa: E402

GIB = 1 << 30
DTYPES = [torch.int8, torch.int16, torch.int32, torch.int64, torch.uint64, torch.float16, torch.bfloat16,
          torch.float32, torch.float64]


def timeit(fn, reps):
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
    a = torch.empty(GIB, dtype=torch.uint8, device="cuda").random_()
    b = torch.empty(GIB, dtype=torch.uint8, device="cuda").random_()
    # 1. dtype x op at 1 GiB per operand
    for dt in DTYPES:
        src, dst = a.view(dt), b.view(dt)
        for op in (H.HcclReduceOp.SUM, H.HcclReduceOp.PROD, H.HcclReduceOp.MAX, H.HcclReduceOp.MIN):
            ts = sorted(timeit(lambda: H.local_reduce(dst, src, op), 5) for _ in range(3))
            t = ts[1]
            print(json.dumps({"table": "dtype_op", "dtype": str(dt).replace("torch.", ""), "op": op.name,
                              "us": round(t * 1e6, 1), "GBps": round(3 * GIB / t / 1e9, 1),
                              "frac_8TBps": round(3 * GIB / t / 8e12, 4)}), flush=True)
    # 2. n-ary fold
    per = 1 << 30
    bufs = [torch.empty(per // 4, dtype=torch.float32, device="cuda").uniform_() for _ in range(16)]
    out = torch.empty_like(bufs[0])
    for n in (2, 3, 4, 8, 16):
        ts = sorted(timeit(lambda: H.local_reduce_n(out, bufs[:n]), 5) for _ in range(3))
        t = ts[1]
        nbytes = (n + 1) * per
        print(json.dumps({"table": "reduce_n", "n": n, "bytes": nbytes, "us": round(t * 1e6, 1),
                          "GBps": round(nbytes / t / 1e9, 1), "frac_8TBps": round(nbytes / t / 8e12, 4)}), flush=True)
    del bufs, out
    # 3. size sweep fp32 SUM
    src, dst = a.view(torch.float32), b.view(torch.float32)
    nbytes = 1 << 10
    while nbytes <= GIB:
        n = nbytes // 4
        reps = 200 if nbytes < (16 << 20) else 10
        ts = sorted(timeit(lambda: H.local_reduce(dst[:n], src[:n]), reps) for _ in range(3))
        t = ts[1]
        print(json.dumps({"table": "size", "bytes_per_operand": nbytes, "us": round(t * 1e6, 2),
                          "GBps": round(3 * nbytes / t / 1e9, 1)}), flush=True)
        nbytes *= 4


if __name__ == "__main__":
    main()
