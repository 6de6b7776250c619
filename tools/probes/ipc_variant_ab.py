"""A/B of the one-sided kernel's block shares and cache policy (r03): HCCL_AMD_IPC_TILE_KIB (0 = one contiguous
window per block; else interleaved tiles) x HCCL_AMD_IPC_NT (non-temporal loads and stores), on a loopback world
(every rank's blocks in one launch on one GPU; each rank driven from its own host thread), two-shot AllReduce fp32
SUM. Variants are interleaved over rounds; per variant the median per-call time (HIP events on rank 0's stream, the
world's launch stream) and its algorithmic rate (n x 2(3n-2)/n x bytes per rank per launch). Every variant's output
is compared bit for bit with the first variant's.
  python tools/ipc_variant_ab.py > gpurun_out/ipc_variant_ab.jsonl
AB_SWEEP = shapes (default: staging size x workgroups per rank), policy (tiles x nt),
staging (uncached vs cached staging memory, one device), fence (barrier fences x workgroups x threads).
The r03 unroll sweep (profiles/r03_ipc_variant_ab_unroll.jsonl) found the fixed 4 vectors in flight best; its
knobs are gone.
"""
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import hccl_amd as H  # noqa: E402

VARIANTS = [(0, 0), (0, 1), (16, 0), (16, 1), (64, 1), (256, 1)]
# second sweep: (staging area MiB, workgroups per rank) with nt loads/stores, contiguous windows
SHAPES = [(128, 128), (128, 256), (512, 128), (512, 256), (512, 512)]
ROUNDS = int(os.environ.get("AB_ROUNDS", "5"))
CALLS = int(os.environ.get("AB_CALLS", "4"))


def run(n, mib, algo=H.Algo.IPC_TWOSHOT):
    dev = torch.device("cuda", 0)
    comms = H.loopback_world(n)
    for c in comms:
        c.set_algo(algo)
    count = (mib << 20) // 4
    g = torch.Generator(device=dev).manual_seed(11 + n)
    xs = [torch.rand(count, device=dev, generator=g) for _ in range(n)]
    ys = [torch.empty_like(x) for x in xs]
    streams = [torch.cuda.Stream() for _ in range(n)]
    pool = ThreadPoolExecutor(n)

    def call():
        list(pool.map(lambda r: comms[r].all_reduce(xs[r], ys[r], H.HcclReduceOp.SUM, streams[r]), range(n)))

    times = {v: [] for v in VARIANTS}
    ok = {v: True for v in VARIANTS}
    ref = None
    for rnd in range(ROUNDS):
        order = VARIANTS[rnd % len(VARIANTS):] + VARIANTS[:rnd % len(VARIANTS)]
        for v in order:
            os.environ["HCCL_AMD_IPC_TILE_KIB"] = str(v[0])
            os.environ["HCCL_AMD_IPC_NT"] = str(v[1])
            call()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(streams[0])
            for _ in range(CALLS):
                call()
            e1.record(streams[0])
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) * 1e3 / CALLS)
            if ref is None:
                ref = [y.clone() for y in ys]
            else:
                ok[v] = ok[v] and all(bool(torch.equal(a, b)) for a, b in zip(ys, ref))
    status = comms[0].ipc_status() & 1
    pool.shutdown()
    for c in comms:
        c.destroy()
    alg = n * 2 * (3 * n - 2) * count * 4 // n
    for v in VARIANTS:
        med = float(np.median(times[v]))
        print(json.dumps({"ranks": n, "mib_per_rank": mib, "algo": algo.name, "tile_kib": v[0], "nt": v[1],
                          "median_us": round(med, 1), "min_us": round(min(times[v]), 1),
                          "max_us": round(max(times[v]), 1), "TBps": round(alg / med / 1e6, 3),
                          "frac": round(alg / med / 1e6 / 8.0, 4), "same_bits": ok[v],
                          "barrier_timeouts": status}), flush=True)


def run_shapes(n, mib, algo=H.Algo.IPC_TWOSHOT):
    """Staging size (rounds per launch) x workgroups per rank: a fresh world per shape (staging is set up per
    communicator), shapes interleaved over rounds."""
    dev = torch.device("cuda", 0)
    count = (mib << 20) // 4
    g = torch.Generator(device=dev).manual_seed(21 + n)
    xs = [torch.rand(count, device=dev, generator=g) for _ in range(n)]
    ys = [torch.empty_like(x) for x in xs]
    streams = [torch.cuda.Stream() for _ in range(n)]
    pool = ThreadPoolExecutor(n)
    os.environ["HCCL_AMD_IPC_TILE_KIB"] = "0"
    os.environ["HCCL_AMD_IPC_NT"] = "1"
    worlds = {}
    for stg, blocks in SHAPES:
        os.environ["HCCL_AMD_IPC_STAGING_MIB"] = str(stg)
        comms = H.loopback_world(n)
        for c in comms:
            c.set_algo(algo)
            c.set_ipc_blocks(blocks)
        list(pool.map(lambda r: comms[r].all_reduce(xs[r], ys[r], H.HcclReduceOp.SUM, streams[r]), range(n)))
        torch.cuda.synchronize()  # the set-up (staging of this size) happens on the first call
        worlds[(stg, blocks)] = comms
    os.environ.pop("HCCL_AMD_IPC_STAGING_MIB")
    times = {k: [] for k in SHAPES}
    ok = {k: True for k in SHAPES}
    ref = None
    for rnd in range(ROUNDS):
        order = SHAPES[rnd % len(SHAPES):] + SHAPES[:rnd % len(SHAPES)]
        for k in order:
            comms = worlds[k]

            def call():
                list(pool.map(lambda r: comms[r].all_reduce(xs[r], ys[r], H.HcclReduceOp.SUM, streams[r]), range(n)))

            call()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(streams[0])
            for _ in range(CALLS):
                call()
            e1.record(streams[0])
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) * 1e3 / CALLS)
            if ref is None:
                ref = [y.clone() for y in ys]
            else:
                ok[k] = ok[k] and all(bool(torch.equal(a, b)) for a, b in zip(ys, ref))
    pool.shutdown()
    alg = n * 2 * (3 * n - 2) * count * 4 // n
    for k in SHAPES:
        comms = worlds[k]
        status = comms[0].ipc_status() & 1
        for c in comms:
            c.destroy()
        med = float(np.median(times[k]))
        print(json.dumps({"ranks": n, "mib_per_rank": mib, "algo": algo.name, "staging_mib": k[0],
                          "blocks_per_rank": k[1], "nt": 1, "median_us": round(med, 1),
                          "min_us": round(min(times[k]), 1), "max_us": round(max(times[k]), 1),
                          "TBps": round(alg / med / 1e6, 3), "frac": round(alg / med / 1e6 / 8.0, 4),
                          "same_bits": ok[k], "barrier_timeouts": status}), flush=True)


# fourth sweep (AB_SWEEP=staging): uncached (the product) vs cached staging memory, loopback world on one device
STAGINGS = ["uncached", "cached"]


def run_staging(n, mib, algo=H.Algo.IPC_TWOSHOT):
    """HCCL_AMD_IPC_STAGING_CACHED = 0 / 1 (read at set-up): one world per memory type, interleaved over rounds."""
    dev = torch.device("cuda", 0)
    count = (mib << 20) // 4
    g = torch.Generator(device=dev).manual_seed(51 + n)
    xs = [torch.rand(count, device=dev, generator=g) for _ in range(n)]
    ys = [torch.empty_like(x) for x in xs]
    streams = [torch.cuda.Stream() for _ in range(n)]
    pool = ThreadPoolExecutor(n)
    worlds = {}
    for k in STAGINGS:
        os.environ["HCCL_AMD_IPC_STAGING_CACHED"] = "1" if k == "cached" else "0"
        comms = H.loopback_world(n)
        for c in comms:
            c.set_algo(algo)
        list(pool.map(lambda r: comms[r].all_reduce(xs[r], ys[r], H.HcclReduceOp.SUM, streams[r]), range(n)))
        torch.cuda.synchronize()
        worlds[k] = comms
    os.environ.pop("HCCL_AMD_IPC_STAGING_CACHED")
    times = {k: [] for k in STAGINGS}
    ok = {k: True for k in STAGINGS}
    ref = None
    for rnd in range(ROUNDS):
        for k in (STAGINGS if rnd % 2 == 0 else STAGINGS[::-1]):
            comms = worlds[k]

            def call():
                list(pool.map(lambda r: comms[r].all_reduce(xs[r], ys[r], H.HcclReduceOp.SUM, streams[r]), range(n)))

            call()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(streams[0])
            for _ in range(CALLS):
                call()
            e1.record(streams[0])
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) * 1e3 / CALLS)
            if ref is None:
                ref = [y.clone() for y in ys]
            else:
                ok[k] = ok[k] and all(bool(torch.equal(a, b)) for a, b in zip(ys, ref))
    pool.shutdown()
    alg = n * 2 * (3 * n - 2) * count * 4 // n
    for k in STAGINGS:
        comms = worlds[k]
        status = comms[0].ipc_status() & 1
        for c in comms:
            c.destroy()
        med = float(np.median(times[k]))
        print(json.dumps({"ranks": n, "mib_per_rank": mib, "algo": algo.name, "staging_memory": k,
                          "median_us": round(med, 1), "min_us": round(min(times[k]), 1),
                          "max_us": round(max(times[k]), 1), "TBps": round(alg / med / 1e6, 3),
                          "frac": round(alg / med / 1e6 / 8.0, 4), "same_bits": ok[k],
                          "barrier_timeouts": status}), flush=True)


# fifth sweep (AB_SWEEP=fence): barrier fences (HCCL_AMD_IPC_LIGHT_FENCE) x workgroups per rank x threads per
# workgroup (HCCL_AMD_IPC_THREADS), one world
FENCES = [(0, 128, 256), (1, 128, 256), (0, 256, 256), (1, 256, 256), (0, 128, 512), (1, 128, 512), (1, 64, 512)]


def run_fence(n, mib, algo=H.Algo.IPC_TWOSHOT):
    """System-scope vs light barrier fences, interleaved over rounds on one world; outputs compared bit for bit."""
    dev = torch.device("cuda", 0)
    comms = H.loopback_world(n)
    for c in comms:
        c.set_algo(algo)
    count = max(64, (mib << 20) // 4)
    g = torch.Generator(device=dev).manual_seed(61 + n)
    xs = [torch.rand(count, device=dev, generator=g) for _ in range(n)]
    ys = [torch.empty_like(x) for x in xs]
    streams = [torch.cuda.Stream() for _ in range(n)]
    pool = ThreadPoolExecutor(n)

    def call():
        list(pool.map(lambda r: comms[r].all_reduce(xs[r], ys[r], H.HcclReduceOp.SUM, streams[r]), range(n)))

    times = {v: [] for v in FENCES}
    ok = {v: True for v in FENCES}
    ref = None
    for rnd in range(ROUNDS):
        order = FENCES[rnd % len(FENCES):] + FENCES[:rnd % len(FENCES)]
        for v in order:
            os.environ["HCCL_AMD_IPC_LIGHT_FENCE"] = str(v[0])
            os.environ["HCCL_AMD_IPC_THREADS"] = str(v[2])
            for c in comms:
                c.set_ipc_blocks(v[1])
            call()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(streams[0])
            for _ in range(CALLS):
                call()
            e1.record(streams[0])
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) * 1e3 / CALLS)
            if ref is None:
                ref = [y.clone() for y in ys]
            else:
                ok[v] = ok[v] and all(bool(torch.equal(a, b)) for a, b in zip(ys, ref))
    os.environ.pop("HCCL_AMD_IPC_LIGHT_FENCE")
    os.environ.pop("HCCL_AMD_IPC_THREADS")
    status = comms[0].ipc_status() & 1
    pool.shutdown()
    for c in comms:
        c.destroy()
    alg = n * 2 * (3 * n - 2) * count * 4 // n
    for v in FENCES:
        med = float(np.median(times[v]))
        print(json.dumps({"ranks": n, "bytes_per_rank": count * 4, "algo": algo.name, "light_fence": v[0],
                          "blocks_per_rank": v[1], "threads": v[2], "median_us": round(med, 1), "min_us": round(min(times[v]), 1),
                          "max_us": round(max(times[v]), 1), "TBps": round(alg / med / 1e6, 3),
                          "frac": round(alg / med / 1e6 / 8.0, 4), "same_bits": ok[v],
                          "barrier_timeouts": status}), flush=True)


def main():
    torch.cuda.set_device(0)
    os.environ.setdefault("HCCL_AMD_IPC_TIMEOUT_MS", "20000")
    if os.environ.get("AB_SWEEP") == "fence":
        for n, mib in ((2, 512), (4, 256), (8, 64)):
            run_fence(n, mib)
    elif os.environ.get("AB_SWEEP") == "staging":
        for n, mib in ((2, 512), (4, 256)):
            run_staging(n, mib)
    elif os.environ.get("AB_SWEEP", "shapes") == "policy":
        for n, mib in ((2, 512), (4, 256), (8, 128)):
            run(n, mib)
    else:
        for n, mib in ((2, 512), (4, 256)):
            run_shapes(n, mib)


if __name__ == "__main__":
    main()
