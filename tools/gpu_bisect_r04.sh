#!/bin/bash
# r04: which earlier tests the hipMemcpyAsync link failure needs (HCCL_AMD_DEVICE_COPY=memcpy, 64 MiB staging):
# subsets of r03's 28-test order ending in the failing test. A time limit or crash ends the call.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out
mkdir -p $OUT
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
ALL=$(python3 -c "print(' '.join(open('tests/r03_failing_selection.txt').read().split()))")
LAST="tests/test_gpu_collectives.py::test_ipc_follows_auto_family[0-4-4099-None]"
sub() { python3 -c "import sys; ids=open('tests/r03_failing_selection.txt').read().split(); print(' '.join([i for i in ids[:-1] if any(k in i for k in sys.argv[1:])] + [ids[-1]]))" "$@"; }
one() {
  local name=$1; shift
  echo "== $name"
  HCCL_AMD_DEVICE_COPY=memcpy HCCL_AMD_IPC_STAGING_MIB=64 timeout -k 10 240 $PYT "$@" > $OUT/bisect_$name.log 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -1 $OUT/bisect_$name.log
  case $rc in 124|137|134|139) echo "stopping"; exit $rc ;; esac
}
one all $ALL
one last_only $LAST
one o2_status $(sub o2_and_status)
one default_staging $(sub default_staging)
one phase_rs_own $(sub phase_trace reduce_scatter_and_reduce ownership)
one no_o2_status $(sub default_staging phase_trace reduce_scatter_and_reduce ownership)
echo done
