# r02: barrier write-back wait + deterministic L2 maintenance: the r01 failure order (maintenance on), the full GPU
# suite, then the IPC size-step probe (one-GPU, 2 ranks)
set -o pipefail
SCRUB=1 RUNS=2 TAG=b bash tools/gpu_seq_ipc.sh && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r02_gpu_suite2.log 2>&1 && \
timeout -k 10 400 python tools/ipc_size_step.py > gpurun_out/r02_ipc_size_step.jsonl 2> gpurun_out/r02_ipc_size_step.err
