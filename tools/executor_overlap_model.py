"""Does the executor's derived synchronisation let the reduce run under the transfers?

The loopback world cannot answer it on one GPU: its links are host-rendezvoused device copies, and its timelines are
host-bound (profiles/r02_overlap_loopback_*.json: the GPU is busy 42-57 % of the span). This tool takes the executor's
own plan instead (HcclAmdExecutorPlan: the units Execute issues, each with its stream and the unit of the other
stream it waits for) for one rank's IR at the C3 shape, and replays it on a two-stream timeline with a cost model:
  link unit    max over peers of the bytes sent to or received from that peer / B_link (76.8 GB/s per direction,
               one xGMI link per peer on a fully connected 8-GPU node);
  reduce unit  algorithmic HBM bytes ((nsrc + 1) x count x elem size per fold, 2 x bytes per copy) / B_hbm (the folds'
               measured 5.7-6.3 TB/s, taken as 6.0 TB/s).
A unit starts when the previous unit of its stream and the unit it waits for have ended (every rank runs the same
plan, so one rank's timeline stands for all). Reported per schedule: link and reduce totals, makespan, the reduce time
that runs while a link unit is in flight (reduce_hidden_frac) and the makespan against the lower bound
max(link total, reduce total); then the makespan again with a launch cost per unit, which prices how many units the
schedule issues: 10 us per transport group plus 1 us per message in it (measured on RCCL self-loop programs,
profiles/r02_rccl_selfloop_latency*.jsonl) and 5 us per fold launch (assumed); and the AllReduce bus bandwidth that
makespan implies (busbw = bytes / makespan x 2(n-1)/n).

  python tools/executor_overlap_model.py > profiles/r02_executor_overlap_model.jsonl
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hccl_amd as H  # noqa: E402

B_LINK = 76.8e9
B_HBM = 6.0e12
# launch cost per unit for the second timeline: a transport group (measured: ~10 us plus ~1 us per message) and a fold
# kernel launch (assumed); it prices the number of units a schedule issues
OVH_LINK = 10e-6
OVH_MSG = 1e-6
OVH_REDUCE = 5e-6


def simulate(ops, nops, es, units, ovh_link=0.0, ovh_reduce=0.0, ovh_msg=0.0):
    end = {0: 0.0, 1: 0.0}
    done = []
    spans = []
    for u in units:
        recs = [ops[i] for i in range(u["first"], u["first"] + u["num"])]
        if u["comm"]:
            per_peer = {}
            for o in recs:
                key = (o.peer, o.kind)
                per_peer[key] = per_peer.get(key, 0) + o.count * es
            dur = max(per_peer.values()) / B_LINK + ovh_link + ovh_msg * len(recs)
        else:
            hbm = 0
            for o in recs:
                hbm += (o.nsrc + 1) * o.count * es if o.kind == H.IrKind.REDUCE else 2 * o.count * es
            dur = hbm / B_HBM + ovh_reduce
        start = end[u["stream"]]
        if u["wait"] >= 0:
            start = max(start, done[u["wait"]])
        fin = start + dur
        end[u["stream"]] = fin
        done.append(fin)
        spans.append((u["stream"], start, fin))
    link = sorted((s, e) for st, s, e in spans if st == 0)
    red = [(s, e) for st, s, e in spans if st == 1]
    hidden = 0.0
    for s, e in red:
        for ls, le in link:
            hidden += max(0.0, min(e, le) - max(s, ls))
    link_total = sum(e - s for s, e in link)
    red_total = sum(e - s for s, e in red)
    makespan = max(done) if done else 0.0
    return {"link_total_ms": round(link_total * 1e3, 3), "reduce_total_ms": round(red_total * 1e3, 3),
            "makespan_ms": round(makespan * 1e3, 3),
            "reduce_hidden_frac": round(hidden / red_total, 3) if red_total else None,
            "makespan_over_bound": round(makespan / max(link_total, red_total), 4) if makespan else None,
            "units": len(units), "link_units": len(link), "reduce_units": len(red)}


def model(op_type, algo, n, count, dtype, rank=0):
    es = H.lib.HcclAmdDataTypeSize(int(dtype))
    ops, nops, used, _ = H.build_schedule(op_type, algo, n, rank, count, dtype)
    units = H.executor_plan(ops, nops, es)
    row = {"op": H.OpType(op_type).name, "algo": H.Algo(used).name, "ranks": n, "bytes_per_rank": count * es}
    row.update(simulate(ops, nops, es, units))
    with_cost = simulate(ops, nops, es, units, OVH_LINK, OVH_REDUCE, OVH_MSG)["makespan_ms"]
    row["makespan_with_launch_cost_ms"] = with_cost
    if op_type == H.OpType.ALLREDUCE and with_cost:
        row["allreduce_busbw_GBps_with_launch_cost"] = round(count * es / (with_cost * 1e-3) * 2 * (n - 1) / n / 1e9, 1)
    return row


CASES = [
    # C3: AllReduce fp32 4 GiB per rank at 8 ranks, every family
    (H.OpType.ALLREDUCE, H.Algo.RING, 8, (4 << 30) // 4, H.HcclDataType.FP32),
    (H.OpType.ALLREDUCE, H.Algo.MESH_CHUNK, 8, (4 << 30) // 4, H.HcclDataType.FP32),
    (H.OpType.ALLREDUCE, H.Algo.MESH_TWOSHOT, 8, (4 << 30) // 4, H.HcclDataType.FP32),
    (H.OpType.ALLREDUCE, H.Algo.RHD, 8, (4 << 30) // 4, H.HcclDataType.FP32),
    (H.OpType.ALLREDUCE, H.Algo.NHR, 8, (4 << 30) // 4, H.HcclDataType.FP32),
    # C4: ReduceScatter bf16, 2 GiB input per rank (recvCount = 128 Mi elements)
    (H.OpType.REDUCE_SCATTER, H.Algo.MESH_CHUNK, 8, (2 << 30) // 2 // 8, H.HcclDataType.BFP16),
    (H.OpType.REDUCE_SCATTER, H.Algo.RING, 8, (2 << 30) // 2 // 8, H.HcclDataType.BFP16),
    # 256 MiB per rank (the loopback timelines' size)
    (H.OpType.ALLREDUCE, H.Algo.MESH_TWOSHOT, 8, (256 << 20) // 4, H.HcclDataType.FP32),
    (H.OpType.ALLREDUCE, H.Algo.MESH_CHUNK, 8, (256 << 20) // 4, H.HcclDataType.FP32),
]


def main():
    for c in CASES:
        print(json.dumps(model(*c)), flush=True)


if __name__ == "__main__":
    main()
