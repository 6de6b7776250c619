#!/bin/bash
# A/B of the IPC staging L2 scrub on the recycled-pages regression test (diagnostics; run under gpurun).
set -uo pipefail
mkdir -p gpurun_out
HCCL_AMD_IPC_L2_SCRUB=0 timeout -k 10 150 python -u -m pytest tests/test_gpu_collectives.py -q --timeout 140 \
    --timeout-method thread -k "recycled" > gpurun_out/t_b0.log 2>&1
echo "scrub off: $(grep -E 'passed|failed' gpurun_out/t_b0.log | tail -1)"
grep -E "AssertionError" gpurun_out/t_b0.log | cut -c1-300 | head -2
timeout -k 10 150 python -u -m pytest tests/test_gpu_collectives.py -q --timeout 140 --timeout-method thread \
    -k "recycled" > gpurun_out/t_b1.log 2>&1
echo "scrub on: $(grep -E 'passed|failed' gpurun_out/t_b1.log | tail -1)"
grep -E "AssertionError" gpurun_out/t_b1.log | cut -c1-300 | head -2
exit 0
