#!/bin/bash
# The GPU-suite order that exposed the stale-staging failure (bootstrap, IPC, executor-loop, auto-family tests), run
# twice with the L2 scrub on (diagnostics; run under gpurun).
set -uo pipefail
mkdir -p gpurun_out
K="bootstrap or o2_and or reduce_scatter_and or ownership or auto_family"
for i in 1 2; do
    timeout -k 10 150 python -u -m pytest tests/test_gpu_bootstrap.py tests/test_gpu_collectives.py -q --timeout 100 \
        --timeout-method thread -k "$K" > gpurun_out/t_seq$i.log 2>&1
    echo "run $i: $(grep -E 'passed|failed' gpurun_out/t_seq$i.log | tail -1)"
    grep -E "AssertionError: rank" gpurun_out/t_seq$i.log | cut -c1-300 | head -2
done
exit 0
