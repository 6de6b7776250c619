"""bench.py's N > 1 entry cannot be misrun: `--gpus N` without a launcher starts the N ranks
itself (torch.distributed.run, one rank per GPU, before any GPU call in the parent) and relays rank 0's line; a
WORLD_SIZE that disagrees with --gpus, or fewer GPUs than ranks, is refused with one JSON line and exit code 6.
These run on the CPU: this container has no GPU, so every real launch here ends in the refusal."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

EXIT_REFUSED = 6


def _run(args, **env):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "HCCL_AMD_BENCH_HOST_EXCHANGE",
              "HCCL_AMD_BENCH_SELFLOOP"):
        e.pop(k, None)
    e.update({k: str(v) for k, v in env.items()})
    e["HIP_VISIBLE_DEVICES"] = e.get("HIP_VISIBLE_DEVICES", "")  # no GPU here either way
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=e,
                       capture_output=True, text=True, timeout=240)
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    return r.returncode, lines, r.stderr


def test_launch_command_is_one_rank_per_gpu_on_this_node():
    cmd = bench.launch_command(8, ["--gpus", "8", "--steps", "3"], 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29555"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"] and cmd[-5].endswith("bench.py")


@pytest.mark.skipif(bench._device_count() > 0, reason="the refusal needs a node with fewer GPUs than asked for")
def test_plain_gpus_8_without_enough_gpus_is_refused_not_a_c2_line():
    rc, lines, err = _run(["--gpus", "8", "--steps", "2", "--warmup", "1"])
    assert rc == EXIT_REFUSED, (rc, lines, err[-2000:])
    assert len(lines) == 1, lines
    line = json.loads(lines[0])
    assert line["n_gpus"] == 8 and line["value"] is None
    assert "GPU" in line["error"]["refused"]
    assert "C2" not in json.dumps(line["config"])


def test_world_size_must_equal_gpus():
    rc, lines, err = _run(["--gpus", "4"], WORLD_SIZE=2, RANK=0, LOCAL_RANK=0)
    assert rc == EXIT_REFUSED, (rc, err[-2000:])
    line = json.loads(lines[0])
    assert "WORLD_SIZE=2 but --gpus 4" in line["error"]["refused"]
    # the other ranks refuse too, silently (rank 0 speaks for the run)
    rc, lines, _ = _run(["--gpus", "4"], WORLD_SIZE=2, RANK=1, LOCAL_RANK=1)
    assert rc == EXIT_REFUSED and lines == []


def test_torchrun_without_gpus_flag_is_refused():
    """`torchrun --nproc-per-node 2 bench.py` (no --gpus: 1 by default) is a mismatch, not an N = 1 line."""
    rc, lines, _ = _run([], WORLD_SIZE=2, RANK=0, LOCAL_RANK=0)
    assert rc == EXIT_REFUSED
    assert json.loads(lines[0])["error"]["refused"].startswith("WORLD_SIZE=2 but --gpus 1")


@pytest.mark.skipif(bench._device_count() > 0, reason="checks the launcher's path on a GPU-less node")
def test_launcher_starts_the_ranks_and_relays_rank0_line():
    """The harness mode allows all ranks on one GPU, so the parent launches: two rank processes start under
    torch.distributed.run, each finds no GPU and refuses, and the parent relays rank 0's single line."""
    rc, lines, err = _run(["--gpus", "2", "--steps", "2", "--warmup", "1"], HCCL_AMD_BENCH_HOST_EXCHANGE=1)
    assert rc != 0, err[-2000:]
    assert "[bench] launching" in err and "torch.distributed.run" in err
    assert len(lines) == 1, (lines, err[-3000:])
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["error"]["world_size_env"] == 2, line


def test_data_path_recommendation_from_rows():
    c3 = {"MESH_CHUNK": {"ms": 20.0, "ran": "MESH_CHUNK"}, "IPC": {"ms": 18.0, "ran": "IPC"},
          "MESH_TWOSHOT": {"ms": 19.0, "ran": "MESH_TWOSHOT"}, "IPC_TWOSHOT": {"error": "x"}}
    pts = []
    for b, auto, dflt, ipc in ((1024, 40.0, 8.0, None), (2048, 41.0, 9.0, None), (1 << 20, 60.0, 30.0, None),
                               (2 << 20, 70.0, None, 90.0), (4 << 20, 80.0, None, 120.0)):
        row = {"bytes": b, "auto_us": auto, "auto_ran": "MESH_ONESHOT"}
        if dflt is not None:
            row.update(auto_default_us=dflt, auto_default_ran="IPC")
        if ipc is not None:
            row.update(ipc_us=ipc, ipc_ran="IPC")
        pts.append(row)
    r = bench.recommend_data_paths(c3, {"points": pts})
    assert r["c3"] == {"mesh_chunk": {"rccl_ms": 20.0, "one_sided_ms": 18.0, "choose": "one_sided"}}
    assert r["c5_ranges"] == [{"from_bytes": 1024, "to_bytes": 1 << 20, "choose": "one_sided"},
                              {"from_bytes": 2 << 20, "to_bytes": 4 << 20, "choose": "rccl"}]
    # a harness line (every row on the one-sided kernel) recommends nothing
    assert bench.recommend_data_paths({"MESH_CHUNK": {"ms": 1.0, "ran": "IPC"}, "IPC": {"ms": 1.0, "ran": "IPC"}},
                                      {"points": [{"bytes": 1024, "auto_us": 5.0, "auto_ran": "IPC"}]}) == \
        {"c3": {}, "c5_ranges": [], "note": r["note"]}
