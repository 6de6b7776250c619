#!/bin/bash
# rocprofv3 evidence for the n-ary fold (the mesh schedules' reduce at 8 GPUs), run on the GPU box from the repo root:
# kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate --pmc passes. Usage: tools/profile_fold.sh r01 8
set -euo pipefail
TAG=${1:-r01}
N=${2:-8}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/prof_fold_$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$REPO/tools/fold_driver.py" "$N" 8
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 "$REPO/tools/fold_driver.py" "$N" 4
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 "$REPO/tools/fold_driver.py" "$N" 4
