"""Device copies and the r03 stale-operand failure (DESIGN.md §5b "Root cause of the stale operands").

r03's driver suite failed in test_ipc_follows_auto_family: a loopback executor fold read zeros for lines of one
operand. The operand was a staging slot filled by the loopback link, a device-to-device hipMemcpyAsync on the
receiver's stream; a host copy after hipDeviceSynchronize still read the slot's old zeros, and only after a later
kernel launch did memory hold the copied bytes. r03's 28-test order with 64 MiB IPC staging reproduced it in every run
with either barrier fence setting (profiles/r04_link_copy_experiment.txt); with the links and the executor's COPY
records done by this library's copy kernel (LaunchCopyBytes, the default) it passed in every run. The regression test
replays that order in a child process, once per fence setting; the copy kernel itself is checked over ragged sizes,
misaligned ends and pointers whose 16-B phases differ.
"""
import ctypes
import os
import subprocess
import sys

import pytest
import torch

import hccl_amd as H

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("fence", ["1", "0"])
def test_r03_failing_order_passes_with_kernel_copies(fence):
    """The r03 failing order (28 tests, ending in the auto run after an IPC call) at 64 MiB staging, in a child
    process so the allocation history is the one that reproduced the failure."""
    ids = open(os.path.join(ROOT, "tests", "r03_failing_selection.txt")).read().split()
    env = dict(os.environ, HCCL_AMD_IPC_STAGING_MIB="64", HCCL_AMD_IPC_LIGHT_FENCE=fence)
    r = subprocess.run([sys.executable, "-u", "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "--timeout", "120",
                        "--timeout-method", "thread", *ids], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-6000:] + r.stderr[-2000:]
    assert f"{len(ids)} passed" in r.stdout, r.stdout[-2000:]


def test_user_copy_at_the_end_of_the_r03_failing_order():
    """a caller's own device-to-device copy (torch copy_, a hipMemcpyAsync) into sendBuf on the
    collective's stream immediately before HcclAllReduce, run at the end of the r03 failing order (the allocation
    history that reproduced the link-copy failure, 64 MiB staging). The library's copies are its kernel; the caller's
    is not, and the fold reads what it wrote."""
    ids = open(os.path.join(ROOT, "tests", "r03_failing_selection.txt")).read().split()
    ids.append("tests/test_gpu_user_copy.py::test_user_copy_then_allreduce")
    env = dict(os.environ, HCCL_AMD_IPC_STAGING_MIB="64")
    r = subprocess.run([sys.executable, "-u", "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "--timeout", "120",
                        "--timeout-method", "thread", *ids], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=400)
    assert r.returncode == 0, r.stdout[-6000:] + r.stderr[-2000:]
    assert f"{len(ids) - 1 + 4} passed" in r.stdout, r.stdout[-2000:]


@pytest.mark.parametrize("nbytes", [1, 15, 16, 17, 4099, (1 << 20) + 5, (64 << 20) + 3])
@pytest.mark.parametrize("shift", [(0, 0), (3, 3), (1, 6), (0, 8), (2, 6), (0, 2), (5, 9)])
def test_device_copy_kernel_bytes(nbytes, shift):
    """LaunchCopyBytes (reached through HcclAmdLocalReduceN with one source, the single-operand fold): every byte
    copied, none outside the range, for aligned, equally misaligned and differently phased pointers (phase differences
    0, 8, 4, 2 and odd: the 16-, 8-, 4-, 2- and 1-byte unit paths)."""
    so, do = shift
    g = torch.Generator(device="cuda").manual_seed(nbytes + 7 * so + do)
    src = torch.randint(0, 256, (nbytes + 32,), dtype=torch.uint8, device="cuda", generator=g)
    dst = torch.full((nbytes + 32,), 0xA5, dtype=torch.uint8, device="cuda")
    s, d = src[so:so + nbytes], dst[do:do + nbytes]
    H.check("HcclAmdLocalReduceN",
            H.lib.HcclAmdLocalReduceN(d.data_ptr(), (ctypes.c_void_p * 1)(s.data_ptr()), 1, nbytes,
                                      int(H.HcclDataType.INT8), int(H.HcclReduceOp.SUM),
                                      torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert torch.equal(d, s)
    host = dst.cpu().numpy()
    assert (host[:do] == 0xA5).all() and (host[do + nbytes:] == 0xA5).all()
