#!/bin/bash
# One parameterised GPU call (replaces r02's one-off gpu_call_r02*.sh recipes). Run on the GPU box from the repo root:
#   tools/gpu_call.sh STEP [STEP ...]        e.g. /usr/local/graft/bin/gpurun -- 'tools/gpu_call.sh rccl_failure host_cost'
# Each step runs under its own time limit and writes gpurun_out/<step>*. An ordinary failure (exit 1) moves on to the
# next step; a time limit (124/137), an abort (134) or a segfault (139) ends the call there: nothing more touches the
# GPU after it. Steps:
#   suite          pytest -m gpu (the round-end suite), smoke, default bench
#   rccl_failure   tests of the RCCL path's failure handling, bootstrap and capture
#   pg             the torch.distributed backend's GPU tests
#   destroy_probe  destroy with a live graph: returns at once, the reaper tears down when the graph goes
#   destroy_probe_immediate  the pre-r03 immediate teardown with a live graph (ends on its limit: run it last)
#   host_cost      host enqueue cost of the RCCL path by category (default, watchdog off, blocking RCCL)
#   ipc_pmc        rocprofv3 kernel trace + FETCH_SIZE + WRITE_SIZE of the one-sided kernel, rank mode, n = 2
#   span_pmc       the same over a self-loop MeshChunk program (RCCL copies + folds)
#   span_channels  self-loop MeshChunk and ring program spans at 0 (RCCL defaults) / 4 / 8 / 16 p2p channels per peer
#   bench          bench.py default line
#   profile        tools/profile_round.sh: rocprofv3 trace + FETCH/WRITE of the N=1 bench line, per-kernel summaries
#   ipc_ab         one-sided kernel: block shares (contiguous / tiles) x cache policy A/B, loopback world
#   harness        bench.py's N > 1 code path with two ranks sharing the GPU (IPC-only; a crash check, not a result)
#   harness_wide   the same with 4 and 8 ranks
#   counters       the TCC counters this rocprofv3 offers
#   ipc_staging    one-sided kernel: uncached vs cached staging memory (A/B on one device)
#   ipc_fence      one-sided kernel: system-scope vs light barrier fences x workgroups per rank (A/B)
#   ipc_system_fence_tests  the one-sided kernel's GPU tests with the system-scope barrier fences
#   ipc_latency_fence  one-sided kernel latency, rank mode, system vs light fences
#   phase_trace_variants  the phase trace with light fences and with cached staging
#   phase_trace    per-block phase stamps of the one-sided two-shot kernel, loopback worlds n = 2, 4, 8
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
REPO=$(pwd)
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp

run() {  # run NAME LIMIT CMD...: stop the call on a time limit, abort or crash
  local name=$1 limit=$2
  shift 2
  echo "== $name (limit ${limit}s)"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"
  tail -5 "$OUT/$name.log"
  case $rc in 124|137|134|139) echo "stopping: $name ended with $rc"; exit $rc ;; esac
  return $rc
}

step_suite() {
  export HCCL_AMD_RANDOM_DRAWS=${HCCL_AMD_RANDOM_DRAWS:-1000}
  run suite 780 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
  run smoke 180 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  step_bench
}

step_rccl_failure() {
  run rccl_failure 600 python3 -u -m pytest tests/test_gpu_rccl_failure.py tests/test_gpu_bootstrap.py \
    tests/test_gpu_rccl.py -v -s --timeout 200 --timeout-method thread -p no:cacheprovider
}

step_pg() {
  run pg 400 python3 -u -m pytest tests/test_gpu_process_group.py -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider
}

step_destroy_probe() {
  run destroy_probe_deferred 60 python3 -u tools/destroy_probe.py
}

# r03 evidence (profiles/r03_destroy_probe_immediate.txt): with the immediate teardown ncclCommFinalize stays in
# progress while the graph lives and ncclCommAbort then blocks too; the step ends on its limit (last in a call).
step_destroy_probe_immediate() {
  HCCL_AMD_DEFER_DESTROY=0 HCCL_EXEC_TIMEOUT=5 run destroy_probe_immediate 40 python3 -u tools/destroy_probe.py
}


step_host_cost() {
  : > "$OUT/host_cost.jsonl"
  HCCL_AMD_HOST_PROFILE=1 run host_cost_default 120 python3 -u tools/host_cost_probe.py
  cat "$OUT/host_cost_default.log" | grep '^{' >> "$OUT/host_cost.jsonl"
  HCCL_AMD_HOST_PROFILE=1 HCCL_AMD_GRAPH_CACHE=0 run host_cost_eager 120 python3 -u tools/host_cost_probe.py
  cat "$OUT/host_cost_eager.log" | grep '^{' >> "$OUT/host_cost.jsonl"
  HCCL_AMD_HOST_PROFILE=1 HCCL_AMD_GRAPH_CACHE=0 HCCL_EXEC_TIMEOUT=0 run host_cost_no_watchdog 120 \
    python3 -u tools/host_cost_probe.py
  cat "$OUT/host_cost_no_watchdog.log" | grep '^{' >> "$OUT/host_cost.jsonl"
  HCCL_AMD_HOST_PROFILE=1 HCCL_AMD_GRAPH_CACHE=0 HCCL_AMD_RCCL_BLOCKING=1 run host_cost_blocking 120 python3 -u tools/host_cost_probe.py
  cat "$OUT/host_cost_blocking.log" | grep '^{' >> "$OUT/host_cost.jsonl"
}

ipc_pmc_one() {  # DTYPE MODE(trace|fetch|write) PORT
  local dt=$1 mode=$2 port=$3
  local args=(--world 2 --mib 512 --dtype "$dt" --algo IPC_TWOSHOT --iters 10 --port "$port")
  local prof
  case $mode in
    trace) prof=(--kernel-trace --stats) ;;
    fetch) prof=(--pmc FETCH_SIZE) ;;
    write) prof=(--pmc WRITE_SIZE) ;;
  esac
  timeout -k 10 150 python3 -u tools/ipc_pmc_rank.py --rank 1 "${args[@]}" > "$OUT/ipc_pmc_${dt}_${mode}_r1.log" 2>&1 &
  local pid1=$!
  run "ipc_pmc_${dt}_${mode}" 150 rocprofv3 "${prof[@]}" --output-format csv -d "$OUT/ipc_pmc_${dt}_${mode}" -o run \
    -- python3 -u tools/ipc_pmc_rank.py --rank 0 "${args[@]}"
  local rc=$?
  wait $pid1
  return $rc
}

step_ipc_pmc() {
  local port=29631
  for dt in fp32 fp16; do
    for mode in trace fetch write; do
      port=$((port + 1))
      ipc_pmc_one "$dt" "$mode" "$port"
    done
  done
}

step_span_pmc() {
  local args=(--algo mesh_chunk --units 64 --iters 5)
  run span_mesh_chunk_trace 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/span_trace" -o run \
    -- python3 -u tools/rccl_selfloop_trace.py "${args[@]}"
  run span_mesh_chunk_fetch 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/span_fetch" -o run \
    -- python3 -u tools/rccl_selfloop_trace.py "${args[@]}"
  run span_mesh_chunk_write 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/span_write" -o run \
    -- python3 -u tools/rccl_selfloop_trace.py "${args[@]}"
}

# r04: the self-loop program span under each per-peer channel setting (0 = RCCL's defaults). On a one-rank self loop
# the per-peer count caps the only "link", so this shows what the xGMI-sized default costs the one-GPU proxy.
step_span_channels() {
  : > "$OUT/span_channels.jsonl"
  local algo v
  for algo in mesh_chunk ring; do
    for v in 0 4 8 16; do
      HCCL_AMD_P2P_CHANNELS_PER_PEER=$v run "span_channels_${algo}_$v" 150 python3 -u tools/rccl_selfloop_trace.py \
        --algo "$algo" --units 64 --iters 5 || return $?
      grep '^{' "$OUT/span_channels_${algo}_$v.log" | python3 -c "import json,sys; [print(json.dumps(dict(json.loads(l), p2p_channels_per_peer_env=$v))) for l in sys.stdin]" >> "$OUT/span_channels.jsonl"
    done
  done
}

step_bench() {
  run bench 300 python3 bench.py
  grep '^{' "$OUT/bench.log" > "$OUT/bench.json" || true
}

step_profile() {
  run profile_round 1000 bash tools/profile_round.sh "${PROFILE_TAG:-r03b}"
}

step_harness() {
  run harness_n2 420 bash tools/gpu_harness_n2.sh
}

# the same with 4 and 8 ranks on the one GPU (every rank's buffers in one HBM: 8 x 8 GiB at N = 8)
step_harness_wide() {
  HARNESS_N=4 HARNESS_LIMIT=600 run harness_n4 620 bash tools/gpu_harness_n2.sh || return $?
  HARNESS_N=8 HARNESS_LIMIT=900 run harness_n8 920 bash tools/gpu_harness_n2.sh
}

step_ipc_ab() {
  run ipc_ab 400 python3 -u tools/ipc_variant_ab.py
  grep '^{' "$OUT/ipc_ab.log" > "$OUT/ipc_variant_ab.jsonl" || true
}

step_ipc_staging() {
  AB_SWEEP=staging run ipc_staging 400 python3 -u tools/ipc_variant_ab.py
  grep '^{' "$OUT/ipc_staging.log" > "$OUT/ipc_variant_ab_staging.jsonl" || true
}

step_ipc_fence() {
  AB_SWEEP=fence run ipc_fence 400 python3 -u tools/ipc_variant_ab.py
  grep '^{' "$OUT/ipc_fence.log" > "$OUT/ipc_variant_ab_fence.jsonl" || true
}

# every one-sided-kernel GPU test with the system-scope barrier fences (HCCL_AMD_IPC_LIGHT_FENCE=0; the rank-mode
# children inherit it; light fences are the default): loopback worlds, rank mode, the random stress
step_ipc_system_fence_tests() {
  HCCL_AMD_IPC_LIGHT_FENCE=0 HCCL_AMD_RANDOM_DRAWS=1000 run ipc_system_fence_tests 600 python3 -u -m pytest \
    tests/test_gpu_ipc_ranks.py tests/test_gpu_ipc_stress.py tests/test_gpu_collectives.py -m gpu -k "ipc or IPC or aiv or AIV" \
    -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
}

# one-sided kernel latency in rank mode (two processes on the GPU), eager and from a graph, system vs light fences
step_ipc_latency_fence() {
  : > "$OUT/ipc_latency_fence.jsonl"
  local port=29561 f
  for f in 0 1 0 1; do
    port=$((port + 1))
    HCCL_AMD_IPC_LIGHT_FENCE=$f run "ipc_latency_fence_$port" 200 python3 -m torch.distributed.run --nnodes=1 \
      --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port tools/graph_latency.py --algo IPC \
      --sizes 1024,65536,1048576,16777216 || return $?
    grep '^{' "$OUT/ipc_latency_fence_$port.log" >> "$OUT/ipc_latency_fence.jsonl" || true
  done
}

step_phase_trace() {
  run phase_trace 300 python3 -u tools/ipc_phase_trace.py
  grep '^{' "$OUT/phase_trace.log" > "$OUT/ipc_phase_trace.jsonl" || true
}

step_phase_trace_variants() {
  HCCL_AMD_IPC_LIGHT_FENCE=1 run phase_trace_light 200 python3 -u tools/ipc_phase_trace.py
  grep '^{' "$OUT/phase_trace_light.log" > "$OUT/ipc_phase_trace_light.jsonl" || true
  HCCL_AMD_IPC_STAGING_CACHED=1 run phase_trace_cached 200 python3 -u tools/ipc_phase_trace.py
  grep '^{' "$OUT/phase_trace_cached.log" > "$OUT/ipc_phase_trace_cached.jsonl" || true
}

step_counters() {
  run counters 60 rocprofv3 -L
  grep -E "TCC_EA0?_(RD|WR)REQ|FETCH_SIZE|WRITE_SIZE" "$OUT/counters.log" | head -60 > "$OUT/counters_tcc.txt" || true
}

for s in "$@"; do
  "step_$s" || echo "step $s: failed (rc=$?), continuing"
done
