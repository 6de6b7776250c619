"""A plain C program on the GPU through the drop-in ABI (tests/c_sample/allreduce_sample.c, built by
__graft_entry__.build()): the reference sample's call sequence with HIP in place of ACL, a one-rank RCCL communicator,
four pthread-driven ranks of a loopback world (AllReduce, ReduceScatter, Reduce) and the inner primitive, every value
checked exactly by the program itself."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

SAMPLE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c_sample", "allreduce_sample")


def test_c_caller_on_the_gpu():
    assert os.path.exists(SAMPLE), "build() did not build the C sample"
    out = subprocess.run([SAMPLE], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and "C SAMPLE OK" in out.stdout, (out.returncode, out.stdout[-2000:], out.stderr[-2000:])
