# r02: full GPU suite, N = 1 bench line, then the N > 1 code path in the one-GPU harness
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r02_gpu_suite3.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r02_bench_n1.json 2> gpurun_out/r02_bench_n1.err && \
bash tools/gpu_harness_n2.sh > gpurun_out/r02_harness.log 2>&1
