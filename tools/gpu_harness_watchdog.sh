#!/bin/bash
# r02: bench.py's N > 1 watchdog in the one-GPU harness: secondary configs stopped at a short deadline (DEADLINE, default 0.5 s) must still print
# the headline line (with "watchdog") and end every rank with EXIT_WATCHDOG (4; r04: failures show in the exit code).
set -uo pipefail
mkdir -p gpurun_out
HCCL_AMD_BENCH_EXTRAS_DEADLINE_S=${DEADLINE:-0.5} HCCL_AMD_BENCH_HOST_EXCHANGE=1 timeout -k 10 300 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 3 --warmup 1 \
    > gpurun_out/bench_harness_watchdog.json 2> gpurun_out/bench_harness_watchdog.err
rc=$?
echo "rc=$rc"
tail -c 600 gpurun_out/bench_harness_watchdog.json
exit $rc
