#!/bin/bash
# r04 experiment on the deterministic repro (the r03 failing selection at 64 MiB staging, light barrier fences):
# control (hipMemcpyAsync links), system-scope barrier fences, and the library's copy kernel for links and copies.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out
mkdir -p $OUT
export HCCL_AMD_DIAG_OUT=$OUT/diag.jsonl
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
SEL=$(python3 -c "print(' '.join(open('tests/r03_failing_selection.txt').read().split()))")
one() {  # one NAME ENV...
  local name=$1; shift
  echo "== $name"
  env HCCL_AMD_IPC_STAGING_MIB=64 "$@" timeout -k 10 240 $PYT $SEL > $OUT/exp_$name.log 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -1 $OUT/exp_$name.log
  case $rc in 124|137|134|139) echo "stopping"; exit $rc ;; esac
}
for i in 1 2; do
  one "memcpy_light_$i" HCCL_AMD_DEVICE_COPY=memcpy HCCL_AMD_IPC_LIGHT_FENCE=1
  one "memcpy_system_$i" HCCL_AMD_DEVICE_COPY=memcpy HCCL_AMD_IPC_LIGHT_FENCE=0
  one "kernel_light_$i" HCCL_AMD_DEVICE_COPY=kernel HCCL_AMD_IPC_LIGHT_FENCE=1
  one "kernel_system_$i" HCCL_AMD_DEVICE_COPY=kernel HCCL_AMD_IPC_LIGHT_FENCE=0
done
echo done
