#!/bin/bash
# r02 round-end rehearsal: what the driver runs at round end (pytest -m gpu, smoke, default bench), on the committed
# tree, each step under its own limit, stopping at the first failure.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export HCCL_AMD_RANDOM_DRAWS=${HCCL_AMD_RANDOM_DRAWS:-1000}
timeout -k 10 780 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/final_gpu_suite.log 2>&1 || { tail -30 gpurun_out/final_gpu_suite.log; echo "gpu suite failed"; exit 1; }
tail -3 gpurun_out/final_gpu_suite.log
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > gpurun_out/final_smoke.log 2>&1 || { tail -30 gpurun_out/final_smoke.log; echo "smoke failed"; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err \
  || { tail -30 gpurun_out/final_bench.err; echo "bench failed"; exit 1; }
cat gpurun_out/final_bench.json
