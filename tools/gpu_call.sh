#!/bin/bash
# GPU-box steps of this round (run from the repo root under gpurun): tools/gpu_call.sh STEP [STEP ...]
#   suite        pytest -m gpu (the driver's suite), then smoke()
#   tests        pytest over the files / ids in $TESTS
#   bench        bench.py default line (N = 1) -> gpurun_out/bench.json
#   profile      tools/profile_round.sh $TAG (rocprofv3 trace + FETCH_SIZE + WRITE_SIZE of the N = 1 line)
#   harness      bench.py's N > 1 path with $HARNESS_N ranks sharing the GPU (IPC-only communicators; a crash check)
#   launcher     bench.py's N > 1 entry on a one-GPU box: a plain --gpus 8 (the refusal, exit 6) and the harness through
#                the launcher (HCCL_AMD_BENCH_HOST_EXCHANGE=1 python3 bench.py --gpus 2: n_gpus 2)
#   selfloop     the RCCL stand-in of the N > 1 line (HCCL_AMD_BENCH_SELFLOOP=1 bench.py --gpus 8: rank 0's programs
#                over a one-rank RCCL self loop, every RCCL-path row)
# Every step runs under its own time limit; a limit, abort or crash ends the call there.
set -o pipefail
REPO=$(pwd)
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp

run() {  # run NAME LIMIT CMD...
  local name=$1 limit=$2
  shift 2
  echo "== $name (limit ${limit}s)"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"
  tail -4 "$OUT/$name.log"
  case $rc in 124|137|134|139) echo "stopping: $name ended with $rc"; exit $rc ;; esac
  return 0
}

step_suite() {
  run suite 900 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider
  run smoke 180 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
}

step_tests() {
  # shellcheck disable=SC2086
  run tests 900 python3 -u -m pytest $TESTS -v --timeout 300 --timeout-method thread -p no:cacheprovider
}

step_bench() {
  echo "== bench"
  timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
  local rc=$?
  echo "   rc=$rc"; cat "$OUT/bench.json"
  case $rc in 124|137|134|139) exit $rc ;; esac
}

step_profile() {
  run profile 1000 bash tools/profile_round.sh "${TAG:-r06}"
}

step_harness() {
  local n=${HARNESS_N:-2}
  echo "== harness n=$n"
  HCCL_AMD_BENCH_HOST_EXCHANGE=1 timeout -k 10 "${HARNESS_LIMIT:-500}" python3 -m torch.distributed.run --nnodes=1 \
    --nproc-per-node "$n" --master-addr 127.0.0.1 --master-port $((29511 + n)) bench.py --gpus "$n" --steps 3 \
    --warmup 1 > "$OUT/bench_harness_n$n.json" 2> "$OUT/bench_harness_n$n.err"
  local rc=$?
  echo "   rc=$rc"; tail -3 "$OUT/bench_harness_n$n.err"
  case $rc in 124|137|134|139) exit $rc ;; esac
}

step_launcher() {
  echo "== launcher: plain --gpus 8 on a one-GPU box"
  timeout -k 10 120 python3 bench.py --gpus 8 > "$OUT/bench_refuse_n8.json" 2> "$OUT/bench_refuse_n8.err"
  local rc=$?
  echo "   rc=$rc (6 = refused)"; cat "$OUT/bench_refuse_n8.json"
  case $rc in 124|137|134|139) exit $rc ;; esac
  echo "== harness through the launcher: python3 bench.py --gpus 2"
  HCCL_AMD_BENCH_HOST_EXCHANGE=1 timeout -k 10 "${HARNESS_LIMIT:-500}" python3 bench.py --gpus 2 --steps 3 --warmup 1 \
    > "$OUT/bench_harness_launcher_n2.json" 2> "$OUT/bench_harness_launcher_n2.err"
  rc=$?
  echo "   rc=$rc"; cut -c1-400 "$OUT/bench_harness_launcher_n2.json"
  case $rc in 124|137|134|139) exit $rc ;; esac
}

step_selfloop() {
  echo "== self-loop stand-in: HCCL_AMD_BENCH_SELFLOOP=1 python3 bench.py --gpus 8"
  HCCL_AMD_BENCH_SELFLOOP=1 timeout -k 10 "${SELFLOOP_LIMIT:-600}" python3 bench.py --gpus 8 --steps 3 --warmup 1 \
    > "$OUT/bench_selfloop_n8.json" 2> "$OUT/bench_selfloop_n8.err"
  local rc=$?
  echo "   rc=$rc"; cut -c1-400 "$OUT/bench_selfloop_n8.json"; tail -3 "$OUT/bench_selfloop_n8.err"
  case $rc in 124|137|134|139) exit $rc ;; esac
}

for s in "$@"; do
  "step_$s"
done
