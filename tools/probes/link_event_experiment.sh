#!/bin/bash
# is r03's stale-operand failure the loopback link's hipMemcpyAsync itself, or the link events'
# lifetime? The loopback transport destroyed its `ready` / `done` events right after another thread's stream had been
# told to wait on them; since r05 it retires them until the world is torn down (comm.cc LoopbackWorld::Retire), and
# HCCL_AMD_LOOPBACK_EVENT_DESTROY=immediate restores the old lifetime. The r03 failing order at 64 MiB staging
# (tests/r03_failing_selection.txt) failed 12 of 12 with hipMemcpyAsync links in r04. Each configuration below runs it
# `REPS` times in a fresh process; the summary line per run goes to gpurun_out/link_event_experiment.txt.
# Usage (GPU box, repo root): tools/probes/link_event_experiment.sh [REPS]
set -uo pipefail
REPS=${1:-2}
OUT=gpurun_out/link_event_${EXPERIMENT:-events}.txt
mkdir -p gpurun_out
: > "$OUT"
IDS=$(cat tests/r03_failing_selection.txt)
run() {  # NAME DEVICE_COPY EVENT_DESTROY [VAR=VALUE ...]: extra environment for the HIP runtime
  local name=$1 copy=$2 destroy=$3 rep rc
  shift 3
  for rep in $(seq 1 "$REPS"); do
    env HCCL_AMD_IPC_STAGING_MIB=64 HCCL_AMD_DEVICE_COPY="$copy" HCCL_AMD_LOOPBACK_EVENT_DESTROY="$destroy" "$@" \
      timeout -k 10 240 python3 -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread $IDS \
      > "gpurun_out/link_event_${name}_${rep}.log" 2>&1
    rc=$?
    echo "$name rep $rep rc $rc: $(tail -1 "gpurun_out/link_event_${name}_${rep}.log")" | tee -a "$OUT"
    # a time limit, abort or crash ends the experiment (a wrong result is rc 1 and is the measurement)
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then return $rc; fi
  done
  return 0
}
case "${EXPERIMENT:-events}" in
  events)
    run memcpy_immediate memcpy immediate && run memcpy_deferred memcpy deferred && run kernel_deferred kernel deferred ;;
  runtime)
    # which part of the HIP runtime's device-to-device copy: the SDMA engines (HSA_ENABLE_SDMA=0 makes the runtime use
    # blit kernels), or the copy's ordering against the next work (AMD_SERIALIZE_COPY=3 waits before and after each copy)
    run memcpy_sdma_off memcpy deferred HSA_ENABLE_SDMA=0 && \
      run memcpy_serialize_copy memcpy deferred AMD_SERIALIZE_COPY=3 && run memcpy_plain memcpy deferred ;;
esac
