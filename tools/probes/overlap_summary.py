"""Summarise a rocprofv3 kernel (+ memory-copy) trace of tools/trace_loopback.py: how much of the reduce-kernel time
runs while link copies are in flight (the two-stream overlap of the executor).

Usage: python tools/overlap_summary.py OUT_DIR [--json out.json]
Reads every *kernel_trace.csv and *memory_copy_trace.csv under OUT_DIR. Reduce kernels: names containing
k_reduce. Link traffic: copy kernels (names containing "copy", case-insensitive) and memory-copy records."""
import argparse
import csv
import glob
import json
import os


def _col(row, *keys):
    for k in row:
        for key in keys:
            if key.lower() == k.lower():
                return row[k]
    return None


def _intervals(paths, pick):
    out = []
    for p in paths:
        with open(p) as f:
            for row in csv.DictReader(f):
                name = _col(row, "Kernel_Name", "Name") or ""
                s, e = _col(row, "Start_Timestamp"), _col(row, "End_Timestamp")
                if s is None or e is None:
                    continue
                cls = pick(name)
                if cls:
                    out.append((cls, int(s), int(e)))
    return out


def _union(iv):
    iv = sorted(iv)
    merged = []
    for s, e in iv:
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    return merged


def _length(m):
    return sum(e - s for s, e in m)


def _intersect(a, b):
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out_dir")
    ap.add_argument("--json")
    ap.add_argument("--link", choices=["copy", "rccl"], default="copy",
                    help="what counts as a link op: device copies and RCCL kernels (loopback world), or only RCCL "
                         "kernels (a real transport, where copies are the schedule's own COPY records)")
    ap.add_argument("--after", help="count only what starts after the last kernel whose name contains this (a marker "
                                    "the traced program launches right before its timed region)")
    a = ap.parse_args()
    kt = glob.glob(os.path.join(a.out_dir, "**", "*kernel_trace.csv"), recursive=True)
    mt = glob.glob(os.path.join(a.out_dir, "**", "*memory_copy_trace.csv"), recursive=True)

    def kpick(name):
        if "k_reduce" in name:
            return "reduce"
        if "nccl" in name.lower() or (a.link == "copy" and "copy" in name.lower()):
            return "link"
        return None

    iv = _intervals(kt, kpick)
    if a.link == "copy":
        iv += [("link", s, e) for _, s, e in _intervals(mt, lambda n: "memcpy")]
    if a.after:
        marks = [s for _, s, _ in _intervals(kt, lambda n: "mark" if a.after in n else None)]
        if marks:
            iv = [x for x in iv if x[1] >= max(marks)]
    red = [(s, e) for c, s, e in iv if c == "reduce"]
    lnk = [(s, e) for c, s, e in iv if c == "link"]
    ur, ul = _union(red), _union(lnk)
    ua = _union(red + lnk)
    span = (max(e for _, _, e in iv) - min(s for _, s, _ in iv)) if iv else 0
    res = {
        "reduce_kernels": len(red), "reduce_busy_us": round(_length(ur) / 1e3, 1),
        "link_ops": len(lnk), "link_busy_us": round(_length(ul) / 1e3, 1),
        "reduce_under_link_us": round(_intersect(ur, ul) / 1e3, 1),
        "reduce_hidden_frac": round(_intersect(ur, ul) / max(1, _length(ur)), 3),
        "span_us": round(span / 1e3, 1),
        # GPU-side work (reduce kernels or link copies) in flight, as a fraction of the span: low means the GPU
        # waited on the host (the loopback transport's per-group rendezvous between the rank threads)
        "gpu_busy_frac": round(_length(ua) / max(1, span), 3),
        "idle_gaps_over_50us": sum(1 for a0, a1 in zip(ua, ua[1:]) if a1[0] - a0[1] > 50000),
        "sources": [os.path.relpath(p, a.out_dir) for p in kt + mt],
    }
    print(json.dumps(res))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
