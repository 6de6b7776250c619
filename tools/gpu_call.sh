#!/bin/bash
# GPU-box steps of this round (run from the repo root under gpurun): tools/gpu_call.sh STEP [STEP ...]
#   suite        pytest -m gpu (the driver's suite), then smoke()
#   tests        pytest over the files / ids in $TESTS
#   bench        bench.py default line (N = 1) -> gpurun_out/bench.json
#   profile      tools/profile_round.sh $TAG (rocprofv3 trace + FETCH_SIZE + WRITE_SIZE of the N = 1 line)
#   harness      bench.py's N > 1 path with $HARNESS_N ranks sharing the GPU (IPC-only communicators; a crash check)
#   latency      small-call latency: rank mode (tools/graph_latency.py, n = 2 and 4, RHD and auto) and loopback worlds
#                (tools/small_call_latency.py)
#   hostcost     tools/host_cost_probe.py over a one-rank RCCL self loop, graph cache on and off
#   rankprobe    tools/probes/ipc_rank_probe.py at 300 MiB without and with the input synchronisation (r03 record)
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
  run profile 1000 bash tools/profile_round.sh "${TAG:-r05}"
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

step_latency() {
  : > "$OUT/small_call_latency_rank_mode.jsonl"
  local n algo port=29631
  for n in 2 4; do
    for algo in RHD AUTO; do
      port=$((port + 1))
      run "graph_latency_${algo}_n$n" 240 env HCCL_AMD_HOST_PROFILE=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
        --master-addr 127.0.0.1 --master-port $port tools/graph_latency.py --algo "$algo" \
        --sizes 1024,16384,131072,1048576
      grep -h '^{' "$OUT/graph_latency_${algo}_n$n.log" >> "$OUT/small_call_latency_rank_mode.jsonl" || true
    done
  done
  run small_call_latency 400 python3 -u tools/small_call_latency.py
  grep -h '^{' "$OUT/small_call_latency.log" > "$OUT/small_call_latency_loopback.jsonl" || true
}

step_hostcost() {
  run hostcost 300 env HCCL_AMD_HOST_PROFILE=1 python3 -u tools/host_cost_probe.py
  run hostcost_nograph 300 env HCCL_AMD_HOST_PROFILE=1 HCCL_AMD_GRAPH_CACHE=0 python3 -u tools/host_cost_probe.py
  grep -h '^{' "$OUT/hostcost.log" "$OUT/hostcost_nograph.log" > "$OUT/host_cost_selfloop.jsonl" || true
}

step_rankprobe() {
  : > "$OUT/rank_probe_sync.jsonl"
  run rank_probe_nosync 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29701 tools/probes/ipc_rank_probe.py --mib 64,300,300,300 --no-sync
  run rank_probe_sync 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29702 tools/probes/ipc_rank_probe.py --mib 64,300,300,300
  grep -h '^{' "$OUT/rank_probe_nosync.log" "$OUT/rank_probe_sync.log" > "$OUT/rank_probe_sync.jsonl" || true
}

for s in "$@"; do
  "step_$s"
done
