"""RCCL send/recv throughput over a one-rank self loop by message shape and by RCCL's p2p channel settings.

The ring and mesh schedules move their data with grouped ncclSend/ncclRecv, one message per peer per step. If one
message's copy (the p2p kernel's channels for that peer) cannot stream faster than a 76.8 GB/s xGMI link, the links
are not the bound. A self loop has no link: its copy is HBM to HBM, so this measures the kernel side only. Each
setting runs in a child process (RCCL reads its environment at communicator creation).

  python tools/rccl_p2p_channels_probe.py > gpurun_out/rccl_p2p_channels.jsonl
"""
import ctypes
import json
import os
import subprocess
import sys
import time

SETTINGS = [
    {},
    {"NCCL_NCHANNELS_PER_PEER": "4"},
    {"NCCL_NCHANNELS_PER_PEER": "8"},
    {"NCCL_NCHANNELS_PER_PEER": "16"},
    {"NCCL_MIN_P2P_NCHANNELS": "32", "NCCL_NCHANNELS_PER_PEER": "8"},
]
SHAPES = [(1, 1 << 30), (7, 146 << 20), (7, 16 << 20), (14, 8 << 20)]  # (messages per group, bytes per message)


class UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


def child():
    import torch
    torch.cuda.set_device(0)
    lib = ctypes.CDLL("librccl.so.1", mode=ctypes.RTLD_GLOBAL)
    for f in ("ncclSend", "ncclRecv"):
        getattr(lib, f).argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                    ctypes.c_void_p]
    lib.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, UniqueId, ctypes.c_int]
    lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(UniqueId)]
    uid = UniqueId()
    assert lib.ncclGetUniqueId(ctypes.byref(uid)) == 0
    comm = ctypes.c_void_p()
    assert lib.ncclCommInitRank(ctypes.byref(comm), 1, uid, 0) == 0
    s = torch.cuda.Stream()
    rows = []
    for msgs, nbytes in SHAPES:
        src = torch.empty(msgs * nbytes, dtype=torch.uint8, device="cuda").random_()
        dst = torch.empty_like(src)

        def group():
            assert lib.ncclGroupStart() == 0
            for m in range(msgs):
                a = ctypes.c_void_p(src.data_ptr() + m * nbytes)
                b = ctypes.c_void_p(dst.data_ptr() + m * nbytes)
                assert lib.ncclSend(a, nbytes, 1, 0, comm, ctypes.c_void_p(s.cuda_stream)) == 0
                assert lib.ncclRecv(b, nbytes, 1, 0, comm, ctypes.c_void_p(s.cuda_stream)) == 0
            assert lib.ncclGroupEnd() == 0

        for _ in range(2):
            group()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        iters = 5
        e0.record(s)
        for _ in range(iters):
            group()
        e1.record(s)
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 1e3 / iters
        ok = bool(torch.equal(src, dst))
        rows.append({"messages": msgs, "bytes_per_message": nbytes, "ms": round(t * 1e3, 3),
                     "GBps_per_message": round(nbytes / t / 1e9, 1), "GBps_total": round(msgs * nbytes / t / 1e9, 1),
                     "ok": ok})
        del src, dst
    print(json.dumps(rows), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child()
        return
    for env in SETTINGS:
        t0 = time.perf_counter()
        try:
            p = subprocess.run([sys.executable, __file__, "--child"], capture_output=True, text=True, timeout=120,
                               env=dict(os.environ, **env))
            lines = [ln for ln in p.stdout.splitlines() if ln.startswith("[")]
            rows = json.loads(lines[-1]) if lines else {"rc": p.returncode, "stderr": p.stderr.splitlines()[-5:]}
        except subprocess.TimeoutExpired:
            rows = {"timeout_s": 120}
        print(json.dumps({"env": env, "rows": rows, "s": round(time.perf_counter() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
