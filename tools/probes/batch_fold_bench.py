"""Batched fold (k_reduceN_batch: the folds of one schedule step in one launch) against a single fold of the same
bytes (k_reduceN), as the executor issues them: programs of REDUCE records only, run on a one-rank communicator through
HcclAmdCommExecute (single stream), timed with HIP events. Shapes: the ring / RHD step (7 segments of 2 operands) and the
MeshChunk piece (7 sub-slices of 8 operands), per-segment sizes from 256 KiB to 16 MiB.

  python tools/batch_fold_bench.py > profiles/r02_batch_fold.jsonl
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    import hccl_amd as H
    from tests.test_gpu_rccl import _ir

    torch.cuda.set_device(0)
    comm = H.comm_init_root_info(1, H.get_root_info(), 0)
    s = torch.cuda.Stream()
    for nsrc in (2, 8):
        for seg_mib in (0.25, 1, 2, 4, 16):
            seg = int(seg_mib * (1 << 20)) // 4
            segs = 7
            # inputs: nsrc operand regions per segment in sendBuf; outputs in recvBuf
            x = torch.rand(segs * nsrc * seg, device="cuda")
            out = torch.empty(segs * seg, device="cuda")
            for batched in (True, False):
                if batched:
                    prog = [_ir(H.IrKind.REDUCE, seg, dst=(1, k * seg),
                                srcs=[(0, (k * nsrc + j) * seg) for j in range(nsrc)]) for k in range(segs)]
                else:  # one fold over all segments' bytes: operand j is a contiguous 7-segment region
                    prog = [_ir(H.IrKind.REDUCE, segs * seg, dst=(1, 0),
                                srcs=[(0, j * segs * seg) for j in range(nsrc)])]
                arr = (H.HcclAmdIrOp * len(prog))(*prog)
                for _ in range(3):
                    comm.execute(arr, len(prog), x, out, H.HcclReduceOp.SUM, True, s)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                iters = 50
                e0.record(s)
                for _ in range(iters):
                    comm.execute(arr, len(prog), x, out, H.HcclReduceOp.SUM, True, s)
                e1.record(s)
                torch.cuda.synchronize()
                t = e0.elapsed_time(e1) / 1e3 / iters
                nbytes = (nsrc + 1) * segs * seg * 4
                print(json.dumps({"operands": nsrc, "segments": segs, "segment_MiB": seg_mib, "batched": batched,
                                  "us": round(t * 1e6, 2), "TBps": round(nbytes / t / 1e12, 3)}), flush=True)
    comm.destroy()


if __name__ == "__main__":
    main()
