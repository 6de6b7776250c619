#!/bin/bash
# rocprofv3 evidence for a round (run on the GPU box from the repo root, under gpurun):
#   1. kernel trace + stats of the default bench command (C2 kernel duration)
#   2. FETCH_SIZE pass, 3. WRITE_SIZE pass (separate --pmc runs; MI355X_MICROARCH.md §rocprofv3)
#   4. kernel + memory-copy timeline of an 8-rank loopback MeshChunk AllReduce (two-stream overlap)
# Outputs under gpurun_out/prof_<tag>; copy the summaries into profiles/ locally. Usage: tools/profile_round.sh r01
set -uo pipefail
TAG=${1:-r01}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$REPO/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > "$OUT/bench_trace.json" || exit $?
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 "$REPO/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > "$OUT/bench_fetch.json" || exit $?
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 "$REPO/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > "$OUT/bench_write.json" || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/loopback" -o run \
    -- python3 "$REPO/tools/trace_loopback.py" > "$OUT/loopback.log" 2>&1 || exit $?
cd "$REPO"
python3 tools/overlap_summary.py "$OUT/loopback" --json "$OUT/overlap.json"
ls -R "$OUT" | head -40
