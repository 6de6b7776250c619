"""Phase timeline of the one-sided kernel (r03): where the time of a two-shot IPC AllReduce goes.

HCCL_AMD_IPC_TRACE=1 makes every block of k_ipc_collective stamp its phases (s_memrealtime, 100 MHz; ipc.h
IpcTraceSlot): round start, phase 0 issued, barrier 1 passed, phase 1 issued, barrier 2 passed, phase 2 issued, exit
(lane 0's stores drained). On a loopback world (every rank's blocks in one launch on one GPU) one launch covers the
whole collective. Per call this prints:
  * the launch span (first entry .. last exit) beside the HIP-event time of the call on rank 0's stream;
  * per phase: the median and p90 over blocks of the per-block duration, and the chip-wide window (first block in ..
    last block out); barriers include their own drain (s_waitcnt vmcnt(0)), the L2 write-back, the flag round trip
    and the wait for the peer block;
  * each phase's algorithmic bytes (whole world) over its chip-wide window, and over the median block duration.
Per rank and input byte the two-shot moves 2(n-1)/n (phase 0: read, store to the owner), 2 (phase 1: read own chunk +
n-1 slots, write out + n-1 results) and 2(n-1)/n (phase 2: copy the results) bytes x S/n ... summed in BYTES below.
  python tools/ipc_phase_trace.py > gpurun_out/ipc_phase_trace.jsonl
"""
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["HCCL_AMD_IPC_TRACE"] = "1"

import numpy as np  # noqa: E402
import torch  # noqa: E402

import hccl_amd as H  # noqa: E402

CALLS = int(os.environ.get("TRACE_CALLS", "5"))
SLOTS = ["entry", "round", "phase0", "barrier1", "phase1", "barrier2", "phase2", "exit"]
TICK_US = 0.01  # s_memrealtime: 100 MHz


def phase_bytes(n: int, s_bytes: int) -> dict:
    """Algorithmic bytes of each phase of a two-shot AllReduce, whole world (n ranks of s_bytes each)."""
    per_rank = {"phase0": 2 * (n - 1) * s_bytes // n, "phase1": 2 * s_bytes, "phase2": 2 * (n - 1) * s_bytes // n}
    return {k: v * n for k, v in per_rank.items()}


def summarize(st: np.ndarray, n: int, blocks: int, s_bytes: int, event_us: float) -> dict:
    a = st[:n, :blocks, :].astype(np.int64)  # [rank][block][slot]
    t0 = a[:, :, 0].min()
    span = (a[:, :, 7].max() - t0) * TICK_US
    out = {"launch_span_us": round(float(span), 1), "event_us": round(event_us, 1)}
    pb = phase_bytes(n, s_bytes)
    seg = [("phase0", 1, 2), ("barrier1", 2, 3), ("phase1", 3, 4), ("barrier2", 4, 5), ("phase2", 5, 6),
           ("drain", 6, 7)]
    for name, i, j in seg:
        d = (a[:, :, j] - a[:, :, i]).reshape(-1) * TICK_US
        win = (a[:, :, j].max() - a[:, :, i].min()) * TICK_US
        row = {"median_us": round(float(np.median(d)), 1), "p10_us": round(float(np.percentile(d, 10)), 1),
               "p90_us": round(float(np.percentile(d, 90)), 1), "max_us": round(float(d.max()), 1),
               "window_us": round(float(win), 1)}
        if name in pb and win > 0:
            row["TBps_over_window"] = round(pb[name] / (win * 1e-6) / 1e12, 3)
            med = float(np.median(d))
            row["TBps_over_median"] = round(pb[name] / (med * 1e-6) / 1e12, 3) if med > 0 else None
        out[name] = row
    # entry skew: how far apart the blocks start (launch fill)
    ent = (a[:, :, 0] - t0).reshape(-1) * TICK_US
    out["entry_skew_us"] = {"median": round(float(np.median(ent)), 2), "max": round(float(ent.max()), 2)}
    return out


def run(n: int, mib: int, blocks: int = 0):
    dev = torch.device("cuda", 0)
    comms = H.loopback_world(n)
    for c in comms:
        c.set_algo(H.Algo.IPC_TWOSHOT)
        if blocks:
            c.set_ipc_blocks(blocks)
    count = (mib << 20) // 4
    g = torch.Generator(device=dev).manual_seed(31 + n)
    xs = [torch.rand(count, device=dev, generator=g) for _ in range(n)]
    ys = [torch.empty_like(x) for x in xs]
    streams = [torch.cuda.Stream() for _ in range(n)]
    pool = ThreadPoolExecutor(n)

    def call():
        list(pool.map(lambda r: comms[r].all_reduce(xs[r], ys[r], H.HcclReduceOp.SUM, streams[r]), range(n)))

    call()  # set-up
    torch.cuda.synchronize()
    rows = []
    for k in range(CALLS):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(streams[0])
        call()
        e1.record(streams[0])
        torch.cuda.synchronize()
        st, b = comms[0].ipc_trace()
        rows.append(summarize(st, n, b, count * 4, e0.elapsed_time(e1) * 1e3))
        rows[-1]["blocks_per_rank"] = b
    status = comms[0].ipc_status() & 1
    pool.shutdown()
    for c in comms:
        c.destroy()
    for k, r in enumerate(rows):
        r.update({"ranks": n, "mib_per_rank": mib, "call": k, "barrier_timeouts": status})
        print(json.dumps(r), flush=True)


def main():
    torch.cuda.set_device(0)
    os.environ.setdefault("HCCL_AMD_IPC_TIMEOUT_MS", "20000")
    for n, mib in ((2, 512), (4, 256), (8, 128)):
        run(n, mib)


if __name__ == "__main__":
    main()
