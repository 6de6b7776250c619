"""pytest configuration: registers the `gpu` marker and makes the in-tree builds available.

`-m "not gpu"` runs everywhere (oracle, golden fixtures, schedules, ABI/export checks, gloo multi-process);
`-m gpu` needs an MI355X and drives libhccl_amd.so through its C ABI.
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _ensure_built():
    lib = os.path.join(ROOT, "hccl_amd", "libhccl_amd.so")
    if not os.path.exists(lib) and shutil.which("hipcc") is not None:
        subprocess.run(["make", "-C", os.path.join(ROOT, "hccl_amd"), "-j8"], check=True,
                       stdout=subprocess.DEVNULL)
    orc = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(orc):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, stdout=subprocess.DEVNULL)


_ensure_built()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct MI355X (gfx950)")
