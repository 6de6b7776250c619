#!/bin/bash
# The GPU-suite order that exposed the stale-staging failure (bootstrap, IPC, executor-loop, auto-family tests), run
# RUNS times (default 2) with HCCL_AMD_IPC_L2_SCRUB=${SCRUB:-1} (diagnostics; run under gpurun). TAG names the logs.
set -uo pipefail
mkdir -p gpurun_out
K="bootstrap or o2_and or reduce_scatter_and or ownership or auto_family"
export HCCL_AMD_IPC_L2_SCRUB=${SCRUB:-1}
for i in $(seq 1 ${RUNS:-2}); do
    timeout -k 10 150 python -u -m pytest tests/test_gpu_bootstrap.py tests/test_gpu_collectives.py -q --timeout 100 \
        --timeout-method thread -k "$K" > gpurun_out/t_seq${TAG:-}$i.log 2>&1
    rc=$?
    echo "run $i (scrub $HCCL_AMD_IPC_L2_SCRUB): rc $rc $(grep -E 'passed|failed' gpurun_out/t_seq${TAG:-}$i.log | tail -1)"
    grep -E "AssertionError: rank|assert len\(bad\)" gpurun_out/t_seq${TAG:-}$i.log | cut -c1-300 | head -2
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi  # a timeout or crash ends the call; a failed test does not
done
exit 0
