"""Which RCCL log subsystem prints the per-peer p2p channel count (r04): a one-rank communicator through the library
with NCCL_DEBUG=INFO and NCCL_DEBUG_SUBSYS=$SUBSYS into a file, then the file's lines that mention channels.
  NCCL_DEBUG_SUBSYS=ALL python3 tools/rccl_init_log_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.makedirs("gpurun_out", exist_ok=True)
path = os.path.abspath("gpurun_out/rccl_init_probe.%p.log")
os.environ["NCCL_DEBUG"] = "INFO"
os.environ.setdefault("NCCL_DEBUG_SUBSYS", "ALL")
os.environ["NCCL_DEBUG_FILE"] = path
import torch  # noqa: E402
import hccl_amd as H  # noqa: E402

torch.cuda.set_device(0)
c = H.comm_init_root_info(1, H.get_root_info(), 0)
print("configured", H.rccl_p2p_channels())
c.destroy()
f = path.replace("%p", str(os.getpid()))
txt = open(f).read() if os.path.exists(f) else ""
print("log bytes", len(txt))
for line in txt.splitlines():
    if "channel" in line.lower() and ("p2p" in line.lower() or "per peer" in line.lower()):
        print(line[-300:])
