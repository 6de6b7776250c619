"""tools/hccl_test (the reference's all_reduce_test workflow) on the host: the binaries exist after build(), the
operator follows the program name, and malformed arguments are refused with the usage text before any HIP call
(no GPU needed). The GPU runs are tests/test_gpu_hccl_test.py."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tools", "hccl_test", "bin")


def _run(tool, *args):
    exe = os.path.join(BIN, tool)
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tools", "hccl_test")], check=True,
                       stdout=subprocess.DEVNULL)
    return subprocess.run([exe, *args], capture_output=True, text=True, timeout=60)


@pytest.mark.parametrize("tool", ["all_reduce_test", "reduce_scatter_test", "reduce_test", "all_gather_test"])
def test_binaries_built_and_named_after_their_operator(tool):
    p = _run(tool, "-z")
    assert p.returncode == 2
    assert f"usage: {os.path.join(BIN, tool)}" in p.stderr


@pytest.mark.parametrize("args", [
    ["-p", "0"],                       # no ranks
    ["-p", "17"],                      # above the 16 the IPC path maps
    ["-b", "1M", "-e", "1K"],          # max below min
    ["-f", "1"],                       # a factor that never grows
    ["-p", "2", "-r", "2"],            # root outside the ranks
    ["-d", "fp8"],                     # no such reduce dtype
    ["-t", "mpi"],                     # no such transport
    ["-b"],                            # flag without its value
])
def test_malformed_arguments_are_refused(args):
    p = _run("all_reduce_test", *args)
    assert p.returncode == 2, (args, p.stdout, p.stderr)
    assert "usage:" in p.stderr
    assert p.stdout == ""
