#!/bin/bash
# The LL form against the staged one-shot (HCCL_AMD_IPC_LL_BYTES=65536 vs 0): rank mode, n = 2 processes on the one
# GPU, tools/graph_latency.py (eager and graph, auto and RHD families) and the phase trace of
# tools/probes/small_call_phase_trace.py. GPU box, repo root: bash tools/probes/ll_latency_ab.sh
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/ll_latency_ab.jsonl
: > "$OUT"
port=29601
for ll in 0 65536; do
  for algo in AUTO RHD; do
    port=$((port + 1))
    HCCL_AMD_IPC_LL_BYTES=$ll HCCL_AMD_HOST_PROFILE=1 timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 \
      --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port tools/graph_latency.py --algo "$algo" \
      --sizes 1024,16384,65536 > gpurun_out/ll_ab_${ll}_${algo}.log 2> gpurun_out/ll_ab_${ll}_${algo}.err || exit $?
    grep -h '^{' gpurun_out/ll_ab_${ll}_${algo}.log | sed "s/^{/{\"ll_bytes\": $ll, /" >> "$OUT"
  done
  port=$((port + 1))
  HCCL_AMD_IPC_LL_BYTES=$ll HCCL_AMD_HOST_PROFILE=1 timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port tools/graph_latency.py --algo AUTO --op rs \
    --sizes 2048,32768,131072 > gpurun_out/ll_ab_${ll}_rs.log 2> gpurun_out/ll_ab_${ll}_rs.err || exit $?
  grep -h '^{' gpurun_out/ll_ab_${ll}_rs.log | sed "s/^{/{\"ll_bytes\": $ll, /" >> "$OUT"
  port=$((port + 1))
  HCCL_AMD_IPC_LL_BYTES=$ll timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $port tools/probes/small_call_phase_trace.py \
    > gpurun_out/ll_trace_${ll}.jsonl 2> gpurun_out/ll_trace_${ll}.err || exit $?
done
