"""Diagnosis of a wrong executor fold on the GPU (r04: VERDICT r03 "What's weak" #1, the stale-operand failures).

When a loopback executor run returns wrong elements, this finds the rank whose REDUCE record wrote them and, for that
record, tells apart the possible causes from the state the failing run left behind:
  * every operand's bytes as memory holds them (hipMemcpy device-to-host), matched against each rank's input;
  * the same REDUCE record run again over the same operands (HcclAmdCommExecute), and once more after a system-scope
    write-back + invalidate of every XCD's L2 (HcclAmdL2Maintain).
Before any of it, every XCD reads each operand (HcclAmdDiagReadByXcc): a stale line an L2 holds shows on that XCD's
workgroups only; data still dirty in one L2 (not yet in memory) shows on the other XCDs.
Memory right and the re-run right: the original fold raced its operand. Memory right, the re-run wrong and the
re-run after the L2 maintenance right: some L2 held stale lines of the operand. Memory wrong: the copy that filled the
operand read or wrote the wrong bytes.
"""
import ctypes
import json
import os

import numpy as np
import torch

import hccl_amd as H
from oracle import oracle as O
from tests._util import to_host

_HIP = None


def _d2h(ptr: int, nbytes: int) -> np.ndarray:
    global _HIP
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so.7")  # the runtime torch loaded (its soname), not a second copy
        _HIP.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _HIP.hipMemcpy.restype = ctypes.c_int
    buf = np.empty(max(1, nbytes // 4), np.uint32)
    rc = _HIP.hipMemcpy(buf.ctypes.data, ptr, nbytes, 2)  # hipMemcpyDeviceToHost
    assert rc == 0, rc
    return buf


def _refold(comm, rec, send, count, stream):
    prog = (H.HcclAmdIrOp * 1)()
    ctypes.memmove(ctypes.byref(prog[0]), ctypes.byref(rec), ctypes.sizeof(H.HcclAmdIrOp))
    out = torch.zeros(count, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    comm.execute(prog, 1, send, out, O.SUM, single_stream=True, stream=stream)
    torch.cuda.synchronize()
    return to_host(O.FP32, out)


def diagnose(comms, op_type, family, xs, count, root, want, outs, sends, recvs, history=None):
    """A JSON-able summary of the wrong fold(s) (fp32 SUM runs); also appended to $HCCL_AMD_DIAG_OUT if set."""
    n = len(comms)
    stream = torch.cuda.Stream()
    report = {"op_type": op_type, "family": family, "n": n, "count": count, "history": history or {},
              "scratch": [hex(c.scratch()[0]) for c in comms],
              "sends": [hex(s.data_ptr()) for s in sends], "recvs": [hex(r.data_ptr()) for r in recvs], "folds": []}
    for r in range(n):
        bad = np.nonzero(outs[r].view(np.uint32) != want[r].view(np.uint32))[0]
        if not len(bad):
            continue
        # the executor's granule: a single-stream call (payload <= 1 MiB) slices by the payload (ops.cc PieceBytesFor)
        payload = count * 4 * (n if op_type == 1 else 1)
        arr, nops, _, _ = H.build_schedule(op_type, family, n, r, count, O.FP32, root,
                                           max(payload, 128) if payload <= (1 << 20) else 0)
        recs = [k for k in range(nops) if arr[k].kind == H.IrKind.REDUCE and arr[k].dstBuf == 1
                and arr[k].dstOff <= bad[0] < arr[k].dstOff + arr[k].count]
        if not recs:
            continue  # the wrong elements reached this rank through a copy of another rank's fold
        rec = arr[recs[0]]
        lo, hi = int(rec.dstOff), int(rec.dstOff + rec.count)
        inrec = bad[(bad >= lo) & (bad < hi)] - lo
        bases = {0: sends[r].data_ptr(), 1: recvs[r].data_ptr(), 2: comms[r].scratch()[0]}
        operands = []
        # first look, before any host copy: every XCD reads each operand against every rank's input (plain loads),
        # then with non-temporal loads against the best-matching rank
        # the very first look: memory as a host copy reads it
        mem0 = [_d2h(bases[rec.srcBuf[j]] + int(rec.srcOff[j]) * 4, int(rec.count) * 4) for j in range(rec.nsrc)]
        xcc_views = []
        exps = [torch.from_numpy(xs[q][lo:hi].copy()).cuda() for q in range(n)]
        torch.cuda.synchronize()
        for j in range(rec.nsrc):
            addr = bases[rec.srcBuf[j]] + int(rec.srcOff[j]) * 4
            best = None
            for q in range(n):
                exp = exps[q]
                badx, zerox = H.diag_read_by_xcc(addr, exp, False, stream)
                if best is None or sum(badx) < sum(best[1]):
                    best = (q, badx, zerox, exp)
            badnt, _ = H.diag_read_by_xcc(addr, best[3], True, stream)
            xcc_views.append({"rank": best[0], "plain_bad_by_xcc": best[1], "plain_zero_by_xcc": best[2],
                              "nt_bad_by_xcc": badnt})
        for j in range(rec.nsrc):
            addr = bases[rec.srcBuf[j]] + int(rec.srcOff[j]) * 4
            mem = _d2h(addr, int(rec.count) * 4)
            ranks = [q for q in range(n) if np.array_equal(mem, xs[q][lo:hi].view(np.uint32))]
            operands.append({"buf": int(rec.srcBuf[j]), "off": int(rec.srcOff[j]), "addr": hex(addr),
                             "matches_rank": ranks, "zero_words_at_bad": int(np.count_nonzero(mem[inrec] == 0)),
                             "mem_wrong_words": int(min((np.count_nonzero(mem != xs[q][lo:hi].view(np.uint32))
                                                         for q in range(n)), default=-1)),
                             "xcc_first_look": xcc_views[j],
                             "first_d2h_zero_words_at_bad": int(np.count_nonzero(mem0[j][inrec] == 0)),
                             "first_d2h_wrong_words": int(min(np.count_nonzero(mem0[j] != xs[q][lo:hi].view(np.uint32))
                                                              for q in range(n)))})
            after = H.diag_read_by_xcc(addr, exps[xcc_views[j]["rank"]], False, stream)[0]
            operands[-1]["plain_bad_by_xcc_after_d2h"] = after
        first = _refold(comms[r], rec, sends[r], count, stream)
        again_bad = int(np.count_nonzero(first[lo:hi].view(np.uint32) != want[r][lo:hi].view(np.uint32)))
        H.l2_maintain(stream)
        second = _refold(comms[r], rec, sends[r], count, stream)
        after_l2_bad = int(np.count_nonzero(second[lo:hi].view(np.uint32) != want[r][lo:hi].view(np.uint32)))
        report["folds"].append({"rank": r, "record": recs[0], "range": [lo, hi], "bad": int(len(inrec)),
                                "bad_first": int(bad[0]), "operands": operands, "refold_bad": again_bad,
                                "refold_after_l2_maintain_bad": after_l2_bad})
        break  # one fold tells the story; the others repeat it
    path = os.environ.get("HCCL_AMD_DIAG_OUT")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(report) + "\n")
    return report
