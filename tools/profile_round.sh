#!/bin/bash
# rocprofv3 evidence for a round's N=1 bench line (run on the GPU box from the repo root, under gpurun):
#   1. kernel trace + stats of the bench command (durations of k_reduce2, the 8-input k_reduceN, k_ipc_collective)
#   2. FETCH_SIZE pass, 3. WRITE_SIZE pass (separate --pmc runs; MI355X_MICROARCH.md §rocprofv3)
#   4. per-kernel summaries (tools/pmc_summary.py) into gpurun_out/prof_<tag>/ -> copy into profiles/ locally.
# Usage: tools/profile_round.sh r03b
set -uo pipefail
TAG=${1:-r03b}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
BENCH=(python3 "$REPO/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-e2e)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- "${BENCH[@]}" \
    > "$OUT/bench_trace.json" || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- "${BENCH[@]}" \
    > "$OUT/bench_fetch.json" || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- "${BENCH[@]}" \
    > "$OUT/bench_write.json" || exit $?
cd "$REPO"
sum() {  # KERNEL_SUBSTRING ALGORITHMIC_BYTES NAME NOTE
  python3 tools/pmc_summary.py --kernel "$1" --stats "$OUT/trace/*kernel_stats.csv" \
    --fetch "$OUT/fetch/*counter_collection.csv" --write "$OUT/write/*counter_collection.csv" \
    --algorithmic-bytes "$2" --out "$OUT/${TAG}_pmc_$3.json" --note "$4"
}
sum "k_reduce2<" 3221225472 local_reduce "C2: dst = src + dst over 2 x 1 GiB fp32, one launch"
sum "k_reduceN<" 9663676416 fold_n8 "8 x 1 GiB fp32 in, 1 GiB out, one ordered fold"
sum "k_ipc_collective" 4294967296 ipc_two_shot \
  "two-shot AllReduce fp32 SUM, 2-rank loopback world in one launch, 512 MiB per rank: 2 x 2(3n-2)/n x 512 MiB"
cp "$OUT/trace/run_kernel_stats.csv" "$OUT/${TAG}_kernel_stats_bench_n1.csv"
cp "$OUT/bench_trace.json" "$OUT/${TAG}_bench_under_rocprof.json"
ls "$OUT"
