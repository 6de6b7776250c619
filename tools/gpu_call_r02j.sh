#!/bin/bash
# r02: host-side latency floor of the executor + RCCL transport for C5-sized programs (one-rank self loop).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
out=gpurun_out/rccl_selfloop_latency${TAG:+_$TAG}.jsonl
: > "$out"
run() { timeout -k 10 120 python3 tools/rccl_selfloop_trace.py "$@" 2>/dev/null | tail -1 >> "$out" || exit 1; }
run --algo mesh_oneshot --count 512 --dtype FP16 --single --iters 2000
run --algo mesh_twoshot --count 512 --dtype FP16 --single --iters 2000
run --algo nhr --count 512 --dtype FP16 --single --iters 2000
run --algo rhd --count 3584 --dtype FP16 --single --iters 2000
run --algo mesh_oneshot --count 524288 --dtype FP16 --single --iters 1000
run --algo mesh_oneshot --count 524288 --dtype FP16 --single --iters 1000 --piece-bytes 0
run --algo rhd --count 458752 --dtype FP16 --single --iters 1000
cat "$out"
