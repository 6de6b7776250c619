"""Device-to-device copy rate: the library's copy kernel (LaunchCopyBytes, reached through a one-operand
HcclAmdLocalReduceN) against hipMemcpyAsync (HCCL_AMD_DEVICE_COPY=memcpy) and torch's copy_, 1 GiB and 16 MiB,
interleaved rounds, HIP events on the launch stream (r04).
  timeout -k 10 200 python3 tools/copy_kernel_probe.py > gpurun_out/copy_kernel.jsonl
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import hccl_amd as H  # noqa: E402


def main():
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    res = {}
    for nbytes in (1 << 30, 16 << 20):
        x = torch.rand(nbytes // 4, device="cuda")
        y = torch.empty_like(x)
        for rnd in range(3):
            for name in ("kernel", "memcpy", "torch"):
                if name == "memcpy":
                    os.environ["HCCL_AMD_DEVICE_COPY"] = "memcpy"
                else:
                    os.environ.pop("HCCL_AMD_DEVICE_COPY", None)
                with torch.cuda.stream(s):
                    evs = [torch.cuda.Event(enable_timing=True) for _ in range(11)]
                    for k in range(11):
                        if k == 1:
                            pass
                        evs[k].record(s)
                        if k == 10:
                            break
                        if name == "torch":
                            y.copy_(x)
                        else:
                            H.local_reduce_n(y, [x], stream=s)
                torch.cuda.synchronize()
                us = sorted(evs[k].elapsed_time(evs[k + 1]) * 1e3 for k in range(1, 10))
                res.setdefault((nbytes, name), []).extend(us)
        os.environ.pop("HCCL_AMD_DEVICE_COPY", None)
        assert torch.equal(x, y)
    for (nbytes, name), us in res.items():
        us.sort()
        med = us[len(us) // 2]
        print(json.dumps({"bytes": nbytes, "copy": name, "median_us": round(med, 2),
                          "GBps_read_plus_write": round(2 * nbytes / med / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
