#!/bin/bash
# the r03 failing order (tests/r03_failing_selection.txt) under each release mode of the IPC
# path's uncached blocks (HCCL_AMD_X_RELEASE: free | scrubfree | sentinel; HCCL_AMD_X_EAGER_SCRATCH: the executor
# staging at communicator creation), RUNS times each, plus the standalone reuse probe. The two switches existed only in
# the r06 experiment builds (commits e05a25c..7cea7f4); the results are profiles/r06_release_experiment.txt.
# Run from the repo root on the GPU box. Logs: gpurun_out/xrel_<mode>_<i>.log, gpurun_out/xrel_probe.jsonl
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
RUNS=${RUNS:-3}
if [ "${PROBE_ITERS:-300}" != 0 ]; then
  timeout -k 10 180 tools/probes/uncached_reuse_probe ${PROBE_ITERS:-300} > $OUT/xrel_probe.jsonl 2> $OUT/xrel_probe.err
  rc=$?
  echo "probe rc=$rc"; cat $OUT/xrel_probe.jsonl
  case $rc in 124|137|134|139) exit $rc ;; esac
fi
for mode in ${MODES:-free scrubfree sentinel}; do
  for i in $(seq 1 "$RUNS"); do
    HCCL_AMD_X_EAGER_SCRATCH=1 HCCL_AMD_X_RELEASE=$mode timeout -k 10 300 python3 -u -m pytest $(cat tests/r03_failing_selection.txt) -q -s \
      --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/xrel_${mode}_$i.log 2>&1
    rc=$?
    echo "$mode run $i rc=$rc: $(tail -1 $OUT/xrel_${mode}_$i.log)"
    case $rc in 124|137|134|139) exit $rc ;; esac
  done
done
exit 0
