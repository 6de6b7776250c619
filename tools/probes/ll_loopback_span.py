"""Device span of one LL launch at n = 2 and n = 8 (r05 late): a loopback world puts every rank's blocks in one launch
on the one GPU, so the launch's phase stamps (HCCL_AMD_IPC_TRACE) give the whole collective's device time, first
block in to last block out, free of the host meeting that bounds a loopback world's per-call time. Per (n, op, size):
the median and p10/p90 over SPAN_SAMPLES calls, each call synchronised and its stamps read back. AllReduce (auto
family's one-shot) and ReduceScatter, fp32 SUM. Compare two libraries by running the copy of this file in each tree.
  python tools/probes/ll_loopback_span.py > gpurun_out/ll_loopback_span.jsonl
"""
import json
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ["HCCL_AMD_IPC_TRACE"] = "1"

import numpy as np  # noqa: E402
import torch  # noqa: E402

import hccl_amd as H  # noqa: E402

SAMPLES = int(os.environ.get("SPAN_SAMPLES", "60"))
TR_ENTRY, TR_EXIT = 0, 7


def call(comms, op, xs, ys, streams):
    def body(r):
        if op == "ar":
            comms[r].all_reduce(xs[r], ys[r], H.HcclReduceOp.SUM, streams[r])
        else:
            comms[r].reduce_scatter(xs[r], ys[r], H.HcclReduceOp.SUM, streams[r])

    th = [threading.Thread(target=body, args=(r,)) for r in range(len(comms))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()


def main():
    torch.cuda.set_device(0)
    for n in (2, 8):
        comms = H.loopback_world(n)
        for c in comms:
            c.set_algo(H.Algo.IPC)
        streams = [torch.cuda.Stream() for _ in range(n)]
        for op in ("ar", "rs"):
            for nbytes in (1 << 10, 1 << 14, 1 << 16):
                elems = nbytes // 4
                xs = [torch.full((elems * (n if op == "rs" else 1),), float(r + 1), device="cuda") for r in range(n)]
                ys = [torch.empty(elems, device="cuda") for _ in range(n)]
                ll0 = comms[0].ipc_ll_launches()
                spans = []
                for i in range(SAMPLES + 5):
                    call(comms, op, xs, ys, streams)
                    tr, blocks = comms[0].ipc_trace()
                    a = tr[:n, :blocks, :].astype(np.int64)
                    if i >= 5:
                        spans.append((a[:, :, TR_EXIT].max() - a[:, :, TR_ENTRY].min()) / 100.0)
                ok = all(bool(torch.all(y == n * (n + 1) / 2).item()) for y in ys)
                print(json.dumps({"n": n, "op": op, "bytes": nbytes, "blocks_per_rank": int(blocks),
                                  "ll_launches": comms[0].ipc_ll_launches() - ll0, "ok": ok,
                                  "span_us_median": round(float(np.median(spans)), 2),
                                  "span_us_p10": round(float(np.percentile(spans, 10)), 2),
                                  "span_us_p90": round(float(np.percentile(spans, 90)), 2)}), flush=True)
        for c in comms:
            c.destroy()


if __name__ == "__main__":
    main()
