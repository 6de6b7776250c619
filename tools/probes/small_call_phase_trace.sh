#!/bin/bash
# tools/probes/small_call_phase_trace.py at n = 2, rank mode's default fences and the light ones (GPU box, repo root).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29561 tools/probes/small_call_phase_trace.py > gpurun_out/small_call_phase_trace.jsonl \
  2> gpurun_out/small_call_phase_trace.err && \
HCCL_AMD_IPC_LIGHT_FENCE=1 timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29562 tools/probes/small_call_phase_trace.py \
  >> gpurun_out/small_call_phase_trace.jsonl 2>> gpurun_out/small_call_phase_trace.err
