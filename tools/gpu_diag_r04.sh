#!/bin/bash
# r04 diagnosis of the stale-operand failure: the diagnosis self-test, then the two test orders
# that failed (r03's 28-test selection, and the driver suite's order up to the auto-family tests), each with the
# failing test's diagnosis written to gpurun_out/diag.jsonl. A time limit, abort or crash ends the call.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out
mkdir -p $OUT
export HCCL_AMD_DIAG_OUT=$OUT/diag.jsonl
run() {
  local name=$1 limit=$2
  shift 2
  echo "== $name"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -3 "$OUT/$name.log"
  case $rc in 124|137|134|139) echo "stopping: $name ended with $rc"; exit $rc ;; esac
  return 0
}
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
run diag_selftest 180 python3 -u tools/diag_selftest.py
SEL=$(python3 -c "print(' '.join(open('tests/r03_failing_selection.txt').read().split()))")
for i in ${DIAG_REPS:-1 2}; do
  run "sel_$i" 240 $PYT $SEL
done
run driver_order 400 $PYT tests/test_gpu_bootstrap.py tests/test_gpu_c_sample.py tests/test_gpu_collectives.py \
  -k "bootstrap or c_sample or o2_and_status or default_staging or phase_trace or barrier_variants or reduce_scatter_and_reduce or ownership or follows_auto"
echo done
