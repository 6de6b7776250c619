"""A few launches of the ordered n-ary fold for rocprofv3 (kernel trace and PMC passes): n inputs of 1 GiB fp32,
out separate. Usage: python3 tools/fold_driver.py [n] [launches]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hccl_amd as H  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    launches = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    torch.cuda.set_device(0)
    bufs = [torch.empty((1 << 30) // 4, device="cuda").uniform_() for _ in range(n + 1)]
    for _ in range(launches):
        H.local_reduce_n(bufs[n], bufs[:n])
    torch.cuda.synchronize()
    print("ok", n, launches)


if __name__ == "__main__":
    main()
