set -o pipefail
export SC_NS=1,2,3,4,8 SC_TRIALS=6 SC_SHAPES="2x1,2x4,1x4"
timeout -k 10 300 python tools/stream_count_probe.py > gpurun_out/r02_stream_count.jsonl 2> gpurun_out/r02_stream_count.err && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "ipc_ranks or ipc_stress or ipc_handles" > gpurun_out/r02_gpu_ipc.log 2>&1
