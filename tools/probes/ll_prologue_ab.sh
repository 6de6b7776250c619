#!/bin/bash
# The LL kernel's prologue and push reworked (r05 late) against the library before (same box, alternating): rank mode,
# n = 2 processes on the one GPU, tools/graph_latency.py (eager and graph, AllReduce auto and RHD, ReduceScatter) and
# the phase trace of tools/probes/small_call_phase_trace.py. The previous library is a worktree of the base commit
# built at ab_old/ (git worktree add ab_old <base>; make -C ab_old/hccl_amd). GPU box, repo root:
#   bash tools/probes/ll_prologue_ab.sh
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/ll_prologue_ab.jsonl
: > "$OUT"
port=29701
for rep in 1 2; do
  for lib in old new; do
    root=.
    [ "$lib" = old ] && root=ab_old
    for algo in AUTO RHD; do
      port=$((port + 1))
      timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port $port $root/tools/graph_latency.py --algo "$algo" --sizes 1024,16384,65536 \
        > gpurun_out/llp_${lib}_${algo}_$rep.log 2> gpurun_out/llp_${lib}_${algo}_$rep.err || exit $?
      grep -h '^{' gpurun_out/llp_${lib}_${algo}_$rep.log | sed "s/^{/{\"lib\": \"$lib\", \"rep\": $rep, /" >> "$OUT"
    done
    port=$((port + 1))
    timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port $port $root/tools/graph_latency.py --algo AUTO --op rs --sizes 2048,32768,131072 \
      > gpurun_out/llp_${lib}_rs_$rep.log 2> gpurun_out/llp_${lib}_rs_$rep.err || exit $?
    grep -h '^{' gpurun_out/llp_${lib}_rs_$rep.log | sed "s/^{/{\"lib\": \"$lib\", \"rep\": $rep, /" >> "$OUT"
  done
done
for lib in old new; do
  root=.
  [ "$lib" = old ] && root=ab_old
  port=$((port + 1))
  timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $port $root/tools/probes/small_call_phase_trace.py \
    > gpurun_out/llp_trace_${lib}.jsonl 2> gpurun_out/llp_trace_${lib}.err || exit $?
done
