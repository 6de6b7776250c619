"""Workload for a rocprofv3 timeline of the executor: an 8-rank loopback-world AllReduce (fp32 SUM, 64 MiB per rank)
in the MeshChunk family the auto selector picks for C3-sized data (forced here), so that the trace shows the link
copies (loopback transport: device-to-device copies on each rank's link stream) and the ordered n-ary reduce kernels
on each rank's reduce stream. Run under rocprofv3 --kernel-trace --memory-copy-trace; summarise with
tools/overlap_summary.py."""
import os
import sys
import threading

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import hccl_amd as H  # noqa: E402


def main():
    # TRACE_MIB per rank (default 64) and TRACE_ALGO (default MESH_CHUNK); HCCL_BUFFSIZE 16 by default (MeshChunk
    # loops of 8 MiB: eight pipelined units per call), set it to 200 for the reference's own loop sizes
    os.environ.setdefault("HCCL_BUFFSIZE", "16")
    n, count = 8, (int(os.environ.get("TRACE_MIB", "64")) << 20) // 4
    algo = H.Algo[os.environ.get("TRACE_ALGO", "MESH_CHUNK")]
    torch.cuda.set_device(0)
    comms = H.loopback_world(n)
    sends = [torch.rand(count, device="cuda") for _ in range(n)]
    recvs = [torch.empty_like(s) for s in sends]
    streams = [torch.cuda.Stream() for _ in range(n)]
    for c in comms:
        c.set_algo(algo)
    torch.cuda.synchronize()

    def body(r):
        for _ in range(int(os.environ.get("TRACE_CALLS", "3"))):
            comms[r].all_reduce(sends[r], recvs[r], H.HcclReduceOp.SUM, streams[r])

    th = [threading.Thread(target=body, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    print("algo", H.Algo(comms[0].last_algo).name, flush=True)
    for c in comms:
        c.destroy()


if __name__ == "__main__":
    main()
