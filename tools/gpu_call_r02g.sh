# r02: ring/RHD schedules after the whole-region gather (GPU parity at small and full size), then the N > 1 bench
# code path in the one-GPU harness (2 ranks, IPC-only communicators: a crash check, not a result)
set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_collectives.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r02_gpu_ring_rhd.log 2>&1 && \
bash tools/gpu_harness_n2.sh > gpurun_out/r02_harness.log 2>&1
