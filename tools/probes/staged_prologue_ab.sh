#!/bin/bash
# The staged one-sided kernel's per-lane flag pointers loaded behind the push instead of before it (r05 late), against
# the library before (a worktree of the base commit built at ab_old/): rank mode, n = 2 processes on the one GPU, the
# LL form off (HCCL_AMD_IPC_LL_BYTES=0) so every call runs the staged kernel; tools/graph_latency.py, eager and graph,
# AllReduce auto family and ReduceScatter, two alternating repetitions. GPU box, repo root:
#   bash tools/probes/staged_prologue_ab.sh
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/staged_prologue_ab.jsonl
: > "$OUT"
port=29801
for rep in 1 2; do
  for lib in old new; do
    root=.
    [ "$lib" = old ] && root=ab_old
    port=$((port + 1))
    HCCL_AMD_IPC_LL_BYTES=0 timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port $port $root/tools/graph_latency.py --algo AUTO \
      --sizes 1024,65536,262144,1048576 > gpurun_out/spa_${lib}_ar_$rep.log 2> gpurun_out/spa_${lib}_ar_$rep.err || exit $?
    grep -h '^{' gpurun_out/spa_${lib}_ar_$rep.log | sed "s/^{/{\"lib\": \"$lib\", \"rep\": $rep, /" >> "$OUT"
    port=$((port + 1))
    HCCL_AMD_IPC_LL_BYTES=0 timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port $port $root/tools/graph_latency.py --algo AUTO --op rs \
      --sizes 2048,131072,1048576 > gpurun_out/spa_${lib}_rs_$rep.log 2> gpurun_out/spa_${lib}_rs_$rep.err || exit $?
    grep -h '^{' gpurun_out/spa_${lib}_rs_$rep.log | sed "s/^{/{\"lib\": \"$lib\", \"rep\": $rep, /" >> "$OUT"
  done
done
