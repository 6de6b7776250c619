"""Host code under AddressSanitizer and UndefinedBehaviorSanitizer (the build's race/safety net is the
IR checks plus sanitizers on host code): tests/sanitize/sched_replay_asan.cc builds every schedule family with
hccl_amd/csrc/schedule.cc and replays it with the oracle's C replayer, with buffers malloc'd at exactly their declared
sizes, so an out-of-range IR offset or any undefined behaviour ends the run. CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="needs gcc/g++")
def test_schedules_and_replay_are_clean_under_asan_ubsan(tmp_path):
    san = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
    oracle_o = tmp_path / "oracle.o"
    subprocess.run(["gcc", "-std=c11", *san, "-c", os.path.join(ROOT, "oracle", "hccl_oracle.c"), "-o", str(oracle_o)],
                   check=True)
    exe = tmp_path / "sched_replay_asan"
    subprocess.run(["g++", "-std=c++17", *san, "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "sanitize", "sched_replay_asan.cc"),
                    os.path.join(ROOT, "hccl_amd", "csrc", "schedule.cc"), str(oracle_o), "-o", str(exe)], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, (out.stdout[-2000:], out.stderr[-4000:])
    assert "failures 0" in out.stdout
