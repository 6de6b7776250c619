#!/bin/bash
# Timeline of the executor on an 8-rank loopback AllReduce (run under gpurun): kernel + memory-copy trace, then the
# reduce/link overlap summary. Usage: tools/trace_loopback.sh TAG  (TRACE_ALGO, TRACE_MIB, TRACE_CALLS, HCCL_BUFFSIZE
# pass through to tools/trace_loopback.py)
set -uo pipefail
TAG=${1:-r01}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/loopback" -o run \
    -- python3 "$REPO/tools/trace_loopback.py" > "$OUT/loopback.log" 2>&1 || exit $?
cd "$REPO"
python3 tools/overlap_summary.py "$OUT/loopback" --json "$OUT/overlap.json"
