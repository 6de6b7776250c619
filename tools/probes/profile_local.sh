#!/bin/bash
# rocprofv3 evidence for the headline kernel (run on the GPU box from the repo root):
#   1. kernel trace + stats of the default bench command
#   2. FETCH_SIZE pass, 3. WRITE_SIZE pass (separate --pmc runs: TCC counter slots, MI355X_MICROARCH.md §rocprofv3)
# then summarise into profiles/<tag>_*.  Usage: tools/profile_local.sh r01
set -euo pipefail
TAG=${1:-r01}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT" "$REPO/profiles"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$REPO/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > "$OUT/bench_trace.json"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 "$REPO/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > "$OUT/bench_fetch.json"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 "$REPO/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > "$OUT/bench_write.json"
cd "$REPO"
# profiles/ is not merged back by gpurun: copy gpurun_out/prof_$TAG/* locally and rerun the summary there
cp "$OUT/trace/run_kernel_stats.csv" "profiles/${TAG}_kernel_stats_local_reduce.csv"
python3 tools/pmc_summary.py --kernel k_reduce2 --stats "$OUT/trace/run_kernel_stats.csv" \
    --fetch "$OUT/fetch/*counter_collection.csv" --write "$OUT/write/*counter_collection.csv" \
    --algorithmic-bytes 3221225472 --out "profiles/${TAG}_pmc_local_reduce.json" \
    --note "bench.py C2 (dst = src + dst, 2 x 1 GiB fp32), default launch config"
