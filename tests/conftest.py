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

# The one-sided kernel's large staging tier has areas of HCCL_BUFFSIZE / 2 (100 MiB) by default; the IPC tests'
# multi-round counts were sized for 128 MiB areas (a chunk wider than one area runs several staging rounds), so the
# suite keeps that size unless a test sets its own (test_gpu_collectives.py::test_ipc_default_staging and
# test_gpu_ipc_ranks.py::test_ipc_rank_mode_default_staging cover the default). Child processes inherit it.
os.environ.setdefault("HCCL_AMD_IPC_STAGING_MIB", "128")
# AllReduces of up to 1 MiB per rank run on the one-sided kernel by default (HCCL_AMD_SMALL_IPC_BYTES, same bits as the
# schedule they stand for). The suite checks the schedules themselves at those sizes, so it turns the rule off unless a
# test sets it (tests/test_gpu_small_ipc.py covers the rule, its bits and its fallbacks).
os.environ.setdefault("HCCL_AMD_SMALL_IPC_BYTES", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct MI355X (gfx950)")
