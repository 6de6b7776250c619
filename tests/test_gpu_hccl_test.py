"""The HCCL performance test tool's workflow (docs/en/build/build.md:184-204: `mpirun -n 8 ./bin/all_reduce_test -b 8K
-e 64M -f 2 -d fp32 -o sum -p 8`, then check_result = success on every line) over libhccl_amd.so, with the
tools/hccl_test binaries built by __graft_entry__.build(). One GPU here: RCCL at one rank, the IPC communicator with
processes sharing the GPU, and the loopback world's threads. Every element of every size is checked by the tool."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tools", "hccl_test", "bin")


@pytest.mark.parametrize("tool,args", [
    ("all_reduce_test", "-b 8K -e 64M -f 2 -d fp32 -o sum -p 1"),
    ("all_reduce_test", "-b 1K -e 16M -f 4 -d fp16 -o sum -p 2 -t ipc"),
    ("all_reduce_test", "-b 1K -e 4M -f 8 -d bf16 -o max -p 4 -t loopback"),
    ("all_reduce_test", "-b 4K -e 1M -f 16 -d fp16 -o sum -p 4 -t loopback -a 12"),
    ("reduce_scatter_test", "-b 64K -e 16M -f 4 -d bf16 -o sum -p 4 -t loopback"),
    ("reduce_scatter_test", "-b 64K -e 4M -f 8 -d fp32 -o min -p 2 -t ipc"),
    ("reduce_test", "-b 8K -e 8M -f 8 -d int32 -o prod -p 2 -r 1 -t ipc"),
    ("reduce_test", "-b 8K -e 8M -f 8 -d fp64 -o sum -p 3 -r 2 -t loopback"),
    ("all_gather_test", "-b 8K -e 16M -f 8 -d int8 -p 8 -t loopback"),
])
def test_hccl_test_workflow(tool, args):
    exe = os.path.join(BIN, tool)
    assert os.path.exists(exe), "tools/hccl_test not built (__graft_entry__.build())"
    env = dict(os.environ, HCCL_AMD_IPC_TIMEOUT_MS="20000")
    p = subprocess.run([exe] + args.split() + ["-n", "5", "-w", "2"], capture_output=True, text=True, timeout=180,
                       env=env)
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", f"hccl_test_{tool}_{abs(hash(args)) % 10000}.txt"), "w") as f:
        f.write(f"{tool} {args}\n{p.stdout}\n{p.stderr}")
    assert p.returncode == 0, p.stdout + p.stderr
    rows = [ln.split() for ln in p.stdout.splitlines() if ln.strip() and ln.split()[0].isdigit()]
    assert rows, p.stdout
    assert all(r[-1] == "success" for r in rows), p.stdout
