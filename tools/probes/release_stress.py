"""r06, DESIGN.md §5b item 5: the r03 order's allocation history in a loop, in one process, to measure how often a
kernel's output loses 512-B pieces when the one-sided path's uncached blocks go back to the runtime after every
destroy (HcclAmdIpcIdleStaging(release=1) of the r06 experiment builds, the pre-pool behaviour) against keeping them
(the default), and against frees of uncached or cached blocks made outside the library. Results:
profiles/r06_release_stress.txt.

Per iteration: loopback worlds of 2, 4 and 8 ranks make one-sided calls (two-shot, the LL form, ReduceScatter) and are
destroyed; then fresh worlds at HCCL_BUFFSIZE=1 run the executor-loop programs of the failing test (Reduce two-shot,
NHR, the one-sided Reduce and the NHR ReduceScatter) on integer-valued data, where every order is exact, so any lost
byte is a wrong element. One JSON line per iteration with the wrong elements per call, their runs and values; a summary
line at the end. Usage: python3 tools/probes/release_stress.py --mode release|keep --seconds 150"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ.setdefault("HCCL_AMD_IPC_STAGING_MIB", "128")  # the suite's setting (tests/conftest.py)
os.environ.setdefault("HCCL_AMD_SMALL_IPC_BYTES", "0")
import hccl_amd as H  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.test_gpu_collectives import AR, RED, RS, collective  # noqa: E402

A = H.Algo


ITER = [0]


def ints(n, count):
    # tagged with the iteration, so a value left over from an earlier iteration is recognisable (exact in fp32: every
    # sum stays below 2^24)
    base = 1000 * (ITER[0] % 1000)
    return [(np.arange(count) % 251 + 7 * r + 1 + base).astype(np.float32) for r in range(n)]


def check(op_type, n, count, root, xs, outs, keep=None):
    total = sum(xs)
    bad = {}
    for r in range(n):
        if op_type == RED and r != root:
            continue
        want = total[r * count:(r + 1) * count] if op_type == RS else total
        idx = np.nonzero(outs[r] != want)[0]
        if len(idx):
            starts = [int(idx[0])] + [int(idx[i]) for i in range(1, len(idx)) if idx[i] != idx[i - 1] + 1]
            # what the wrong values are: a sum over a subset of this iteration's operands (an operand read stale or
            # missed), a value of an earlier iteration (tag 1000 per iteration), or neither
            off = r * count if op_type == RS else 0
            kinds = {"subset": 0, "earlier_iteration": 0, "other": 0}
            for i in idx[:2000]:
                got = float(outs[r][i])
                ops = [float(x[off + i]) for x in xs]
                if any(abs(got - sum(ops[q] for q in range(n) if m >> q & 1)) < 0.5 for m in range(1 << n)):
                    kinds["subset"] += 1
                elif got < float(want[i]) - 500 * n:
                    kinds["earlier_iteration"] += 1
                else:
                    kinds["other"] += 1
            bad[r] = {"wrong": int(len(idx)), "runs": len(starts), "first_runs": starts[:6],
                      "zeros": int(np.count_nonzero(outs[r][idx] == 0)), "kinds_of_first_2000": kinds,
                      "got_want_first": [float(outs[r][idx[0]]), float(want[idx[0]])]}
            if keep is not None:
                bad[r]["addr"] = {"send": keep["send_ptrs"][r], "recv": keep["recv_ptrs"][r],
                                  "scratch": keep.get("scratch", [None] * n)[r]}
    return bad


_HIP = []


def hip():
    if not _HIP:
        import ctypes
        h = ctypes.CDLL("libamdhip64.so.7")  # the runtime torch loaded
        h.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
        h.hipFree.argtypes = [ctypes.c_void_p]
        h.hipDeviceSynchronize.argtypes = []
        _HIP.append(h)
    return _HIP[0]


def ext_churn(flags):
    """Outside the library: allocate blocks of the sizes the one-sided path frees (its 128 MiB x 4 tier and the 4 MiB +
    32 KiB flags + LL block) with hipExtMallocWithFlags(flags), write them with a kernel (the library's local reduce:
    non-temporal loads and stores over the whole block), synchronise and free them."""
    import ctypes
    h = hip()
    s = torch.cuda.Stream()
    for nbytes in (512 << 20, (4 << 20) + (32 << 10)):
        p = ctypes.c_void_p(0)
        assert h.hipExtMallocWithFlags(ctypes.byref(p), nbytes, flags) == 0
        H.check("HcclAmdLocalReduce", H.lib.HcclAmdLocalReduce(p.value, p.value, nbytes // 4,
                                                                int(H.HcclDataType.INT32), int(H.HcclReduceOp.SUM),
                                                                s.cuda_stream))
        assert h.hipDeviceSynchronize() == 0
        assert h.hipFree(p.value) == 0


def release(mode):
    torch.cuda.synchronize()
    if mode.startswith("release"):
        # the library's own release (r06 experiment builds up to 39bb417; the library now refuses it, NOT_SUPPORT)
        import ctypes
        b = ctypes.c_uint64(0)
        rc = H.lib.HcclAmdIpcIdleStaging(1, ctypes.byref(b))
        if rc != 0:
            raise SystemExit("this library does not release its uncached blocks (HcclAmdIpcIdleStaging: %d)" % rc)
    if mode == "release_wait":  # the same, then time for anything the runtime does after a free
        torch.cuda.synchronize()
        time.sleep(0.05)
    if mode == "keep_ext_uncached":
        ext_churn(0x3)  # hipDeviceMallocUncached
    if mode == "keep_ext_cached":
        ext_churn(0x0)  # hipDeviceMallocDefault


def iteration(mode):
    res = []
    # one-sided calls on worlds that are then destroyed: their uncached blocks go back (release) or stay (keep)
    for n, count in ((2, 37748747), (4, 1000003), (8, 4099)):
        comms = H.loopback_world(n)
        try:
            for algo, op_type, c in ((A.IPC_TWOSHOT, AR, count), (A.IPC, AR, 3000), (A.IPC_TWOSHOT, RS, 5001)):
                xs = ints(n, c * n if op_type == RS else c)
                _, outs = collective(comms, op_type, algo, O.FP32, O.SUM, xs, c)
                b = check(op_type, n, c, 0, xs, outs)
                if b:
                    res.append({"call": f"ipc n={n} algo={algo.name} op={op_type} count={c}", "bad": b})
        finally:
            torch.cuda.synchronize()
            for cm in comms:
                cm.destroy()
        release(mode)
    # the executor-loop programs of test_ownership_orders_follow_executor_loops at HCCL_BUFFSIZE=1
    os.environ["HCCL_BUFFSIZE"] = "1"
    try:
        for op_type, algo, n, count in ((RED, 2, 3, 300001), (RED, 5, 5, 600001), (AR, 5, 6, 700001),
                                        (RED, 7, 4, 300001), (RED, 7, 3, 250003), (RS, 5, 3, 200003)):
            comms = H.loopback_world(n)
            try:
                root = 1
                xs = ints(n, count * n if op_type == RS else count)
                keep = {}
                used, outs = collective(comms, op_type, algo, O.FP32, O.SUM, xs, count, root=root, keep=keep)
                keep["scratch"] = [hex(cm.scratch()[0]) for cm in comms]
                b = check(op_type, n, count, root, xs, outs, keep)
                if b:
                    res.append({"call": f"loops op={op_type} algo={A(used).name} n={n} count={count}", "bad": b})
            finally:
                torch.cuda.synchronize()
                for cm in comms:
                    cm.destroy()
            release(mode)
    finally:
        os.environ.pop("HCCL_BUFFSIZE", None)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=("release", "keep", "release_wait", "keep_ext_uncached", "keep_ext_cached"),
                    default="release")
    ap.add_argument("--seconds", type=float, default=150)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    t0 = time.time()
    it = fails = 0
    while time.time() - t0 < a.seconds:
        ITER[0] = it
        res = iteration(a.mode)
        it += 1
        fails += bool(res)
        print(json.dumps({"probe": "release_stress", "mode": a.mode, "iter": it, "wrong_calls": res}), flush=True)
    print(json.dumps({"probe": "release_stress", "mode": a.mode, "summary": True, "iterations": it,
                      "iterations_with_wrong_calls": fails, "seconds": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
