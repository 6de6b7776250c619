#!/bin/bash
# A/B of the executor events' system-scope fence (HCCL_AMD_EXECUTOR_EVENT_FENCE=0) over the one-rank RCCL self-loop programs
# of tools/host_cost_probe.py, with the executor graph cache on and off. Usage (GPU box, repo root):
#   bash tools/probes/executor_event_fence_ab.sh
set -o pipefail
mkdir -p gpurun_out
export HCCL_AMD_HOST_PROFILE=1 TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/host_cost_probe.py > gpurun_out/fence_default.jsonl 2> gpurun_out/fence_default.err && \
HCCL_AMD_EXECUTOR_EVENT_FENCE=0 timeout -k 10 300 python3 -u tools/host_cost_probe.py > gpurun_out/fence_off.jsonl 2> gpurun_out/fence_off.err && \
HCCL_AMD_GRAPH_CACHE=0 timeout -k 10 300 python3 -u tools/host_cost_probe.py > gpurun_out/fence_default_nograph.jsonl 2>> gpurun_out/fence_default.err && \
HCCL_AMD_GRAPH_CACHE=0 HCCL_AMD_EXECUTOR_EVENT_FENCE=0 timeout -k 10 300 python3 -u tools/host_cost_probe.py > gpurun_out/fence_off_nograph.jsonl 2>> gpurun_out/fence_off.err
