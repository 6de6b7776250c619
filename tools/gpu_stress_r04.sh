#!/bin/bash
# r04: the r03 failing selection under several staging sizes (different allocation layouts), light barrier fences
# (HCCL_AMD_IPC_LIGHT_FENCE=1), each failure diagnosed into gpurun_out/diag.jsonl. A time limit or crash ends the call.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out
mkdir -p $OUT
export HCCL_AMD_DIAG_OUT=$OUT/diag.jsonl
export HCCL_AMD_IPC_LIGHT_FENCE=${HCCL_AMD_IPC_LIGHT_FENCE:-1}
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
SEL=$(python3 -c "print(' '.join(open('tests/r03_failing_selection.txt').read().split()))")
for mib in ${STRESS_MIB:-64 128 256 512 1000 128 512}; do
  echo "== staging $mib MiB"
  HCCL_AMD_IPC_STAGING_MIB=$mib timeout -k 10 240 $PYT $SEL > $OUT/stress_$mib.log 2>&1
  rc=$?
  echo "   rc=$rc"; tail -1 $OUT/stress_$mib.log
  case $rc in 124|137|134|139) echo "stopping"; exit $rc ;; esac
done
echo done
