"""Executor graph replay against eager execution, by payload, for the RCCL-path programs (r06): rank 0's 8-rank
programs over a one-rank RCCL self loop (HcclAmdCommInitSelfLoop), fp32 SUM AllReduce, each size timed with the graph
cache on (the key's third call on replays one captured graph) and off (every call eager). One JSON line per (algo, size).
Usage: python3 tools/graph_crossover.py [--algos RING,MESH_CHUNK] [--mib 1,8,64,256,1024,4096]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hccl_amd as H  # noqa: E402


def timed(call, iters, s):
    for _ in range(3):  # eager, capture, first replay
        call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        call()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--algos", default="RING,MESH_CHUNK,RHD")
    ap.add_argument("--mib", default="1,8,64,256,1024,4096")
    ap.add_argument("--n", type=int, default=8)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()  # the HCCL entries reject the null stream
    sizes = [int(m) for m in a.mib.split(",")]
    x = torch.empty((max(sizes) << 20) // 4, device="cuda").uniform_()
    y = torch.empty_like(x)
    for name in a.algos.split(","):
        for mib in sizes:
            comm = H.comm_init_selfloop(a.n, 0)
            try:
                comm.set_algo(H.Algo[name])
                cnt = (mib << 20) // 4
                xs, ys = x[:cnt], y[:cnt]
                row = {"probe": "graph_crossover", "algo": name, "n": a.n, "mib": mib}
                iters = 20 if mib <= 64 else 5
                for key, cache in (("graph_us", 16), ("eager_us", 0)):
                    comm.set_config(H.Config.GRAPH_CACHE, cache)
                    row[key] = round(timed(lambda: comm.all_reduce(xs, ys, H.HcclReduceOp.SUM, s), iters, s), 1)
                row["ran"] = H.Algo(comm.last_algo).name
                row["graph_launches"], row["graph_captures"] = comm.graph_stats()
                print(json.dumps(row), flush=True)
            finally:
                torch.cuda.synchronize()
                comm.destroy()


if __name__ == "__main__":
    main()
