"""Summarise rocprofv3 output for one kernel into profiles/ JSON.

Usage: python tools/pmc_summary.py --kernel k_reduce2 --stats DIR/run_kernel_stats.csv \
           --fetch DIR_F/..._counter_collection.csv --write DIR_W/..._counter_collection.csv \
           --algorithmic-bytes 3221225472 --out profiles/r01_pmc_local_reduce.json

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB and are collected in
separate passes (TCC slots); on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced streaming
read, so the read side is doubled: hbm = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
"""
import argparse
import csv
import glob
import hashlib
import json
import os
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def library_sha256(path=os.path.join(ROOT, "hccl_amd", "libhccl_amd.so")):
    """Identity of the library the counters were taken on: bench.py compares it with the library it loads, so a
    counter figure taken on other kernels is flagged in the line."""
    try:
        with open(path, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()
    except OSError:
        return None


def counter_values(path, kernel, name):
    vals = []
    for p in glob.glob(path):
        with open(p) as f:
            for row in csv.DictReader(f):
                if kernel in row.get("Kernel_Name", "") and row.get("Counter_Name") == name:
                    vals.append(float(row["Counter_Value"]))
    return vals


def stats_row(path, kernel):
    for p in glob.glob(path):
        with open(p) as f:
            for row in csv.DictReader(f):
                if kernel in row["Name"]:
                    return row
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--stats", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--algorithmic-bytes", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    fetch = counter_values(a.fetch, a.kernel, "FETCH_SIZE")
    write = counter_values(a.write, a.kernel, "WRITE_SIZE")
    st = stats_row(a.stats, a.kernel)
    f_kib = statistics.median(fetch) if fetch else None
    w_kib = statistics.median(write) if write else None
    hbm = (2 * f_kib + w_kib) * 1024 if fetch and write else None
    out = {
        "kernel": st["Name"] if st else a.kernel,
        "launches_traced": int(st["Calls"]) if st else None,
        "avg_duration_ns": float(st["AverageNs"]) if st else None,
        "min_duration_ns": float(st["MinNs"]) if st else None,
        "max_duration_ns": float(st["MaxNs"]) if st else None,
        "fetch_size_kib_raw_median": f_kib,
        "write_size_kib_median": w_kib,
        "pmc_dispatches": {"fetch": len(fetch), "write": len(write)},
        "hbm_bytes_per_launch": hbm,
        "algorithmic_bytes_per_launch": a.algorithmic_bytes,
        "traffic_over_algorithmic": (hbm / a.algorithmic_bytes) if hbm else None,
        "correction": "hbm = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE counts half of a 16 B/lane stream)",
        "note": a.note,
        # provenance: the library profiled and the source commit it was built from (HCCL_AMD_SOURCE_COMMIT, passed in
        # by the GPU call: the GPU box has no .git)
        "library_sha256": library_sha256(),
        "source_commit": os.environ.get("HCCL_AMD_SOURCE_COMMIT"),
    }
    if st:
        out["achieved_GBps_from_trace"] = a.algorithmic_bytes / (float(st["AverageNs"]) * 1e-9) / 1e9
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
