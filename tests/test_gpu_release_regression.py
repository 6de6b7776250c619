"""Regression test for DESIGN.md §5b correctness record item 5: the one-sided path never frees its uncached blocks.

tools/probes/release_stress.py replays the r03 order's allocation history in a loop (loopback worlds making one-sided
calls and being destroyed, then the executor-loop programs of test_ownership_orders_follow_executor_loops on
integer-valued data). With the blocks freed after every destroy, 17 of 217 iterations returned wrong results and runs
ended in memory aperture faults (profiles/r06_release_stress.txt); with the library's default (blocks kept and reused)
223 of 223 were exact. This runs the default for 20 s (about 25 iterations, where a return of the frees would show in
most runs) in a child process and requires every iteration exact."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(180)
def test_loop_of_the_r03_allocation_history_is_exact():
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "probes", "release_stress.py"), "--mode",
                        "keep", "--seconds", "20"], cwd=ROOT, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    summary = lines[-1]
    assert summary.get("summary") and summary["iterations"] >= 5, summary
    wrong = [ln for ln in lines[:-1] if ln["wrong_calls"]]
    assert not wrong, json.dumps(wrong[:3])[:3000]
