#!/bin/bash
# One GPU-box pass (run from the repo root under gpurun): the GPU parity suite, smoke(), the N=1 bench line.
# Every GPU step has its own time limit; the first failure ends the script.
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -4 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { echo "gpu tests rc=$rc"; exit $rc; }
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || exit $?
cat gpurun_out/bench_n1.json
