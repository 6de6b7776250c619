#!/bin/bash
# N>1 code path of bench.py on the one-GPU box: HARNESS_N ranks (default 2) share the GPU over the IPC-only
# communicator (HCCL_AMD_BENCH_HOST_EXCHANGE=1; the RCCL rows report NOT_SUPPORT there). Not a result: a crash check.
set -uo pipefail
mkdir -p gpurun_out
N=${HARNESS_N:-2}
HCCL_AMD_BENCH_HOST_EXCHANGE=1 timeout -k 10 ${HARNESS_LIMIT:-400} python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node "$N" --master-addr 127.0.0.1 --master-port $((29511 + N)) bench.py --gpus "$N" --steps 3 --warmup 1 \
    > gpurun_out/bench_harness_n$N.json 2> gpurun_out/bench_harness_n$N.err
rc=$?
tail -5 gpurun_out/bench_harness_n$N.err
cat gpurun_out/bench_harness_n$N.json
exit $rc
