"""HBM traffic of every kernel after a trace marker, per program, against the program's algorithmic bytes and the HBM
roofline (the one-sided kernel, and the fold + RCCL copy bytes of a self-loop program span).

  python tools/span_pmc_summary.py --fetch 'DIR_F/**/*counter_collection.csv' --write 'DIR_W/**/*counter_collection.csv' \
      --trace 'DIR_T/**/*kernel_trace.csv' --marker FillFunctor --iters 5 --algorithmic-bytes B --out profiles/x.json

Counters (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE in KiB, separate passes; gfx950's FETCH_SIZE counts
half the bytes of a wide (16 B/lane) streaming read, so reads are reported raw and doubled. Dispatches are taken after
the last dispatch whose name holds --marker (by Dispatch_Id) and divided by --iters. The span time is the kernel
trace's first start to last end after the marker, per program.
"""
import argparse
import csv
import glob
import json
from collections import defaultdict


def _rows(pattern):
    for p in glob.glob(pattern, recursive=True):
        with open(p) as f:
            yield from csv.DictReader(f)


def _after_marker(rows, marker, key="Dispatch_Id"):
    rows = sorted(rows, key=lambda r: int(r.get(key) or r.get("Correlation_Id") or 0))
    last = -1
    for i, r in enumerate(rows):
        if marker in (r.get("Kernel_Name") or ""):
            last = i
    return rows[last + 1:]


def counter_by_kernel(pattern, name, marker):
    rows = [r for r in _rows(pattern) if r.get("Counter_Name") == name]
    per = defaultdict(float)
    launches = defaultdict(int)
    for r in _after_marker(rows, marker):
        k = (r.get("Kernel_Name") or "?").split("(")[0][:80]
        per[k] += float(r["Counter_Value"])
        launches[k] += 1
    return per, launches


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--trace", default="")
    ap.add_argument("--marker", default="FillFunctor")
    ap.add_argument("--iters", type=int, required=True)
    ap.add_argument("--algorithmic-bytes", type=int, required=True)
    ap.add_argument("--peak-TBps", type=float, default=8.0)
    ap.add_argument("--label", default="")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fetch, fl = counter_by_kernel(a.fetch, "FETCH_SIZE", a.marker)
    write, _ = counter_by_kernel(a.write, "WRITE_SIZE", a.marker)
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, 0.0) * 1024 / a.iters
        w = write.get(k, 0.0) * 1024 / a.iters
        kernels[k] = {"launches_per_program": fl.get(k, 0) / a.iters, "fetch_bytes_raw": round(f),
                      "fetch_bytes_x2": round(2 * f), "write_bytes": round(w)}
    f_raw = sum(v["fetch_bytes_raw"] for v in kernels.values())
    w_all = sum(v["write_bytes"] for v in kernels.values())
    out = {"label": a.label, "iters": a.iters, "algorithmic_bytes_per_program": a.algorithmic_bytes,
           "hbm_bytes_per_program_fetch_x2": round(2 * f_raw + w_all),
           "hbm_bytes_per_program_fetch_raw": round(f_raw + w_all),
           "traffic_over_algorithmic_x2": round((2 * f_raw + w_all) / a.algorithmic_bytes, 4),
           "traffic_over_algorithmic_raw": round((f_raw + w_all) / a.algorithmic_bytes, 4),
           "kernels": kernels}
    if a.trace:
        rows = _after_marker(list(_rows(a.trace)), a.marker, key="Dispatch_Id")
        if rows:
            t0 = min(int(r["Start_Timestamp"]) for r in rows)
            t1 = max(int(r["End_Timestamp"]) for r in rows)
            span_ns = (t1 - t0) / a.iters
            busy = defaultdict(float)
            for r in rows:
                busy[(r.get("Kernel_Name") or "?").split("(")[0][:80]] += (int(r["End_Timestamp"]) -
                                                                            int(r["Start_Timestamp"])) / a.iters
            out["span_ns_per_program"] = round(span_ns)
            out["kernel_busy_ns_per_program"] = {k: round(v) for k, v in busy.items()}
            out["algorithmic_TBps_over_span"] = round(a.algorithmic_bytes / span_ns / 1e3, 3)
            out["hbm_TBps_over_span_x2"] = round(out["hbm_bytes_per_program_fetch_x2"] / span_ns / 1e3, 3)
            out["frac_of_peak_algorithmic"] = round(out["algorithmic_TBps_over_span"] / a.peak_TBps, 4)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
