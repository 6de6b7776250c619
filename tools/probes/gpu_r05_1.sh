set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/probes/ipc_import_probe > gpurun_out/ipc_import_probe.jsonl 2> gpurun_out/ipc_import_probe.err && \
timeout -k 10 900 python3 -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_small_ipc.py tests/test_gpu_user_copy.py tests/test_gpu_ipc_ranks.py tests/test_gpu_link_copy.py \
  "tests/test_gpu_rccl.py::test_executor_graph_cache_eviction_while_in_flight" \
  "tests/test_gpu_rccl.py::test_rccl_p2p_channels_configured" > gpurun_out/r05_gpu1_tests.log 2>&1; \
rc=$?; echo "pytest rc $rc"; tail -30 gpurun_out/r05_gpu1_tests.log; \
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then timeout -k 10 600 bash tools/probes/link_event_experiment.sh 2; fi
