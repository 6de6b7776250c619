# r02: full GPU suite, then the default bench line (N = 1)
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r02_gpu_suite.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r02_bench_n1.json 2> gpurun_out/r02_bench_n1.err
