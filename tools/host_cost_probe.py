"""Host cost of the RCCL path, one GPU, one-rank RCCL communicator (self loop).

Programs (rank 0's program of an 8-rank schedule, peers mapped onto the self loop; tests/test_gpu_rccl.py self_looped):
  ring7m   the 8-rank ring AllReduce at 7 MiB fp32 (two-stream executor; tools/rccl_soak.py's program); with the
           executor graph cache on (default) the timed calls replay one captured graph, with HCCL_AMD_GRAPH_CACHE=0
           every call is eager
  oneshot  C5's 1 KiB fp16 AllReduce, one-shot (single-stream: one transport group + one 8-input fold)
  group1k  the one-shot's transport group alone (7 sends + 7 receives of 128 B): RCCL's own enqueue cost
  rhd1k / rhd1m  C5's schedule, the 8-rank RHD AllReduce fp16 at 1 KiB and 1 MiB (single-stream: 6 transport groups and
           the halving folds); since r05 single-stream programs replay from the executor graph cache too (the key's
           second call on), so with the cache on the "eager" loop is graph launches
For each: eager wall time per program (enqueue + GPU, K back-to-back programs then one sync), host enqueue time per
program (the loop without the sync), the same program replayed from a HIP graph, and with HCCL_AMD_HOST_PROFILE=1 the
executor's host time by category.
  HCCL_AMD_HOST_PROFILE=1 python tools/host_cost_probe.py > gpurun_out/host_cost.jsonl
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import hccl_amd as H  # noqa: E402
from tests.test_gpu_rccl import self_looped  # noqa: E402

ITERS = int(os.environ.get("PROBE_ITERS", "300"))


def group_only(arr, nops):
    keep = [arr[i] for i in range(nops) if arr[i].kind in (H.IrKind.SEND, H.IrKind.RECV)]
    first = keep[0].group
    keep = [o for o in keep if o.group == first]
    return (H.HcclAmdIrOp * len(keep))(*keep), len(keep)


def measure(comm, name, arr, nops, x, y, single, s, dtype):
    for _ in range(20):
        comm.execute(arr, nops, x, y, H.HcclReduceOp.SUM, single, s, dtype=dtype)
    torch.cuda.synchronize()
    H.host_profile(reset=True)
    t0 = time.perf_counter()
    for _ in range(ITERS):
        comm.execute(arr, nops, x, y, H.HcclReduceOp.SUM, single, s, dtype=dtype)
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    prof = H.host_profile(reset=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        comm.execute(arr, nops, x, y, H.HcclReduceOp.SUM, single, torch.cuda.current_stream(), dtype=dtype)
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(ITERS):
        g.replay()
    torch.cuda.synchronize()
    t_graph = time.perf_counter() - t0
    del g
    groups = len({arr[i].group for i in range(nops) if arr[i].kind in (H.IrKind.SEND, H.IrKind.RECV)})
    out = {"program": name, "graph_cache": os.environ.get("HCCL_AMD_GRAPH_CACHE", "16"),
           "graph_stats_launches_captures": comm.graph_stats(), "records": nops, "groups": groups, "single_stream": single, "iters": ITERS,
           "eager_us": round(t_all / ITERS * 1e6, 2), "enqueue_us": round(t_enq / ITERS * 1e6, 2),
           "graph_us": round(t_graph / ITERS * 1e6, 2),
           "host_us_by_category": {k: round(ns / ITERS / 1e3, 2) for k, (ns, _) in prof.items() if ns},
           "calls_per_program": {k: round(c / ITERS, 2) for k, (_, c) in prof.items() if c},
           "env": {k: v for k, v in os.environ.items() if k.startswith(("HCCL_", "NCCL_", "RCCL_"))}}
    print(json.dumps(out), flush=True)


def main():
    torch.cuda.set_device(0)
    comm = H.comm_init_root_info(1, H.get_root_info(), 0)
    s = torch.cuda.Stream()
    count = 7 * 8 * 64 * 512
    arr, nops, _ = self_looped(H.OpType.ALLREDUCE, int(H.Algo.RING), 8, 0, count, H.HcclDataType.FP32)
    x = torch.rand(count, device="cuda")
    y = torch.empty_like(x)
    measure(comm, "ring7m", arr, nops, x, y, False, s, H.HcclDataType.FP32)
    c5 = 512  # 1 KiB fp16
    arr, nops, _ = self_looped(H.OpType.ALLREDUCE, int(H.Algo.MESH_ONESHOT), 8, 0, c5, H.HcclDataType.FP16)
    xh = torch.rand(c5, device="cuda").half()
    yh = torch.empty_like(xh)
    measure(comm, "oneshot1k", arr, nops, xh, yh, True, s, H.HcclDataType.FP16)
    garr, gn = group_only(arr, nops)
    measure(comm, "group1k", garr, gn, xh, yh, True, s, H.HcclDataType.FP16)
    for name, cnt in (("rhd1k", 512), ("rhd1m", 1 << 19)):
        arr, nops, _ = self_looped(H.OpType.ALLREDUCE, int(H.Algo.RHD), 8, 0, cnt, H.HcclDataType.FP16)
        xr = torch.rand(cnt, device="cuda").half()
        yr = torch.empty_like(xr)
        measure(comm, name, arr, nops, xr, yr, True, s, H.HcclDataType.FP16)
    comm.destroy()


if __name__ == "__main__":
    main()
