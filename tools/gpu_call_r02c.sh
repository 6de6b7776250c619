# r02: AIV-engine orders on the GPU (loopback world + rank mode)
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_collectives.py -m gpu -x -q --timeout 300 --timeout-method thread -k "aiv" > gpurun_out/r02_gpu_aiv.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_ipc_ranks.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_gpu_aiv_ranks.log 2>&1
