#!/bin/bash
# r04: which earlier tests the hipMemcpyAsync link failure needs (HCCL_AMD_DEVICE_COPY=memcpy, 64 MiB staging unless
# STAGING is set): subsets of r03's 28-test order ending in the failing test (profiles/r04_link_copy_bisect.txt).
# A time limit or crash ends the call.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out
mkdir -p $OUT
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
ALL=$(python3 -c "print(' '.join(open('tests/r03_failing_selection.txt').read().split()))")
LAST="tests/test_gpu_collectives.py::test_ipc_follows_auto_family[0-4-4099-None]"
sub() {  # the failing test preceded by the earlier tests whose id contains any of the arguments
  python3 -c "import sys; ids=open('tests/r03_failing_selection.txt').read().split(); print(' '.join([i for i in ids[:-1] if any(k in i for k in sys.argv[1:])] + [ids[-1]]))" "$@"
}
without() {  # the six ownership tests but one, then the failing test
  python3 -c "import sys; ids=open('tests/r03_failing_selection.txt').read().split(); print(' '.join([i for i in ids[:-1] if 'ownership' in i and sys.argv[1] not in i] + [ids[-1]]))" "$1"
}
one() {
  local name=$1; shift
  echo "== $name"
  HCCL_AMD_DEVICE_COPY=memcpy HCCL_AMD_IPC_STAGING_MIB=${STAGING:-64} timeout -k 10 240 $PYT "$@" > $OUT/bisect_$name.log 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -1 $OUT/bisect_$name.log
  case $rc in 124|137|134|139) echo "stopping"; exit $rc ;; esac
}
case ${BISECT_STAGE:-1} in
1)
  one all $ALL
  one last_only $LAST
  one o2_status $(sub o2_and_status)
  one default_staging $(sub default_staging)
  one phase_rs_own $(sub phase_trace reduce_scatter_and_reduce ownership)
  one no_o2_status $(sub default_staging phase_trace reduce_scatter_and_reduce ownership) ;;
2)  # after stage 1: phase_trace + reduce_scatter_and_reduce + ownership suffice
  one phase $(sub phase_trace)
  one rs $(sub reduce_scatter_and_reduce)
  one own $(sub ownership)
  one phase_rs $(sub phase_trace reduce_scatter_and_reduce)
  one phase_own $(sub phase_trace ownership)
  one rs_own $(sub reduce_scatter_and_reduce ownership)
  for k in 0-5-6 2-7-4 2-7-3 1-5-3 2-2-3 2-5-5; do one own_$k $(sub "ownership_orders_follow_executor_loops[$k"); done ;;
3)  # after stage 2: the six ownership tests (each a world created and destroyed) suffice, none alone
  one own_last $(sub ownership)
  HCCL_AMD_TEST_SKIP_IPC_RUN=1 one own_last_no_ipc_run $(sub ownership)
  STAGING=128 one own_last_staging128 $(sub ownership)
  for k in 0-5-6 2-7-4 2-7-3 1-5-3 2-2-3 2-5-5; do one own_minus_$k $(without "[$k"); done ;;
4)  # the whole order, with and without the last test's IPC call
  for i in 1 2; do
    one all_$i $ALL
    HCCL_AMD_TEST_SKIP_IPC_RUN=1 one all_no_ipc_run_$i $ALL
  done ;;
esac
echo done
