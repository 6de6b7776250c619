#!/bin/bash
# N>1 code path of bench.py on the one-GPU box: two ranks share the GPU over the IPC-only communicator
# (HCCL_AMD_BENCH_HOST_EXCHANGE=1; the RCCL rows report NOT_SUPPORT there). Not a result: a crash check.
set -uo pipefail
mkdir -p gpurun_out
HCCL_AMD_BENCH_HOST_EXCHANGE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 \
    > gpurun_out/bench_harness_n2.json 2> gpurun_out/bench_harness_n2.err
rc=$?
tail -5 gpurun_out/bench_harness_n2.err
cat gpurun_out/bench_harness_n2.json
exit $rc
