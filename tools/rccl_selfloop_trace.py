"""Reduce/transfer overlap of the executor with real RCCL kernels on one GPU (hardware side).

One rank's program of an n-rank schedule, its peers mapped onto a one-rank RCCL communicator (tests/test_gpu_rccl.py
self_looped), runs through HcclAmdCommExecute: the RCCL send/recv kernels of every group on the link stream and the
folds on the reduce stream, with the waits the executor derives. Under `rocprofv3 --kernel-trace`,
tools/overlap_summary.py then reports how much fold time runs while an RCCL kernel is in flight and how busy the GPU
is over the span. The self-loop "links" are HBM copies, not xGMI, so the link/fold time ratio is not the 8-GPU one;
what the trace shows is whether the two streams run concurrently on hardware.

  rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rsl -o rsl -- python tools/rccl_selfloop_trace.py --algo ring
  python tools/overlap_summary.py gpurun_out/rsl --link rccl --after FillFunctor --json profiles/r02_overlap_rccl_selfloop_ring.json
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--algo", default="ring")
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--units", type=int, default=64, help="count = 7 * 8 * 64 * 512 * units fp32 elements")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--count", type=int, default=0, help="elements (overrides --units)")
    ap.add_argument("--dtype", default="FP32")
    ap.add_argument("--single", action="store_true", help="the single-stream executor mode (payloads <= 1 MiB)")
    ap.add_argument("--piece-bytes", type=int, default=-1,
                    help="pipelining granule; default: what a collective call uses (the payload when --single)")
    a = ap.parse_args()
    import torch
    import hccl_amd as H
    from tests.test_gpu_rccl import self_looped

    algo = H.Algo[a.algo.upper()]
    count = a.count or 7 * 8 * 64 * 512 * a.units
    dt = H.HcclDataType[a.dtype.upper()]
    es = H.lib.HcclAmdDataTypeSize(int(dt))
    piece = a.piece_bytes if a.piece_bytes >= 0 else (max(count * es, 128) if a.single else 0)
    prog = self_looped(H.OpType.ALLREDUCE, int(algo), a.ranks, a.rank, count, dt, piece)
    if prog is None:
        raise SystemExit("this schedule's groups do not pair up over a self loop at this count")
    arr, nops, _ = prog
    torch.cuda.set_device(0)
    comm = H.comm_init_root_info(1, H.get_root_info(), 0)
    tdt = {"FP32": torch.float32, "FP16": torch.float16, "BFP16": torch.bfloat16}[a.dtype.upper()]
    x = torch.rand(count, device="cuda").to(tdt)
    out = torch.empty_like(x)
    s = torch.cuda.Stream()
    comm.execute(arr, nops, x, out, H.HcclReduceOp.SUM, a.single, s)  # warm-up: RCCL connections, staging
    torch.cuda.synchronize()
    torch.empty(1, device="cuda").fill_(7.0)  # trace marker (a FillFunctor kernel): overlap_summary.py --after Fill
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        comm.execute(arr, nops, x, out, H.HcclReduceOp.SUM, a.single, s)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    comm.destroy()
    groups = len({arr[i].group for i in range(nops) if arr[i].kind in (H.IrKind.SEND, H.IrKind.RECV)})
    # HBM bytes the program must move on this one GPU: a self send/recv pair of B bytes is an RCCL copy (read B,
    # write B); a fold of k inputs reads k and writes 1 operand; a copy reads and writes its bytes
    copy_b = sum(2 * arr[i].count * es for i in range(nops) if arr[i].kind == H.IrKind.SEND)
    fold_b = sum((arr[i].nsrc + 1) * arr[i].count * es for i in range(nops) if arr[i].kind == H.IrKind.REDUCE)
    dcopy_b = sum(2 * arr[i].count * es for i in range(nops) if arr[i].kind == H.IrKind.COPY)
    print(json.dumps({"algo": algo.name, "ranks": a.ranks, "rank": a.rank, "dtype": a.dtype.upper(),
                      "bytes_per_rank": count * x.element_size(), "records": nops, "groups": groups,
                      "single_stream": a.single, "piece_bytes": piece, "us_per_program": round(dt * 1e6, 1),
                      "iters": a.iters, "algorithmic_bytes_per_program": {"rccl_copies": copy_b, "folds": fold_b,
                                                                          "copies": dcopy_b,
                                                                          "total": copy_b + fold_b + dcopy_b}}),
          flush=True)


if __name__ == "__main__":
    main()
