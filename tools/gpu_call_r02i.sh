#!/bin/bash
# r02: executor overlap with real RCCL kernels over a one-rank self loop (tools/rccl_selfloop_trace.py), per schedule.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for algo in ring mesh_chunk mesh_twoshot rhd; do
  rm -rf "gpurun_out/rsl_$algo"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/rsl_$algo" -o rsl -- \
    python3 tools/rccl_selfloop_trace.py --algo "$algo" > "gpurun_out/rsl_$algo.log" 2>&1 || { tail -20 "gpurun_out/rsl_$algo.log"; exit 1; }
  tail -1 "gpurun_out/rsl_$algo.log"
  python3 tools/overlap_summary.py "gpurun_out/rsl_$algo" --link rccl --after FillFunctor --json "gpurun_out/overlap_rccl_selfloop_$algo.json" || exit 1
done
