#!/bin/bash
# r02: IPC_RHD latency beside the IPC auto family and the IPC two-shot, rank mode (n processes share the one GPU;
# not an xGMI measurement), eager and from a HIP graph.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
out=gpurun_out/ipc_rhd_latency.jsonl
: > "$out"
port=29561
for n in 2 4 8; do
  for algo in IPC_RHD IPC IPC_TWOSHOT; do
    port=$((port + 1))
    timeout -k 10 120 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $port tools/graph_latency.py --algo $algo --sizes 1024,65536,1048576,8388608 \
      >> "$out" 2> gpurun_out/ipc_rhd_latency_n${n}_${algo}.err || { echo "failed n=$n $algo"; exit 1; }
  done
done
cat "$out"
