#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X-native HCCL reduce path.

Metric (BASELINE.json): "device-resident reduce GiB/s (fp32 sum) vs HBM peak; ring all-reduce bus GB/s".

  N = 1  (default): config C2 — the local reduce primitive HcclAmdLocalReduce (dst = src + dst, the hcomm
         HcommLocalReduceOnThread replacement) over two 1 GiB fp32 buffers already resident in HBM.
         A step = one launch over the whole 2 x 1 GiB pair; bytes per step = 3 GiB (read src, read dst, write dst).
         value = GiB/s = 3 GiB x K / timed region.
  N > 1  (torchrun, one process per GPU): config C3 — HcclAllReduce fp32 SUM, 4 GiB per rank, over the RCCL
         communicator built from HcclGetRootInfo / HcclCommInitRootInfo. A step = one AllReduce.
         value = whole-job reduced input GiB/s = N x 4 GiB x K / max-over-ranks time; bus GB/s is reported beside it.
         The headline schedule is the ring (BASELINE.json's "ring all-reduce"): HCCL_AMD_ALGO_RING, 7 arc-disjoint
         rings at n = 8; the reference's own selection (MeshChunk) and the other families are extra rows.

Every run prints exactly one JSON line on rank 0 (extra diagnostics go to stderr).
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import platform
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# RCCL's per-peer p2p channels for the N > 1 run: the library sets them only when asked (HCCL_AMD_P2P_CHANNELS_PER_PEER,
# read when it is loaded, i.e. now; comm.cc ConfigureRcclP2pChannels). The bench asks for 16 per peer, the setting r04
# chose on the one-GPU proxy (4 made the self-loop RCCL programs 1.7-2.9x slower, profiles/r04_span_channels.jsonl);
# they apply to torch.distributed's RCCL communicators of this process too. transport.p2p_channels reports what RCCL's
# INIT log says it set up. A caller's own setting wins.
os.environ.setdefault("HCCL_AMD_P2P_CHANNELS_PER_PEER", "16")

import hccl_amd as H  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md "Chip-level parameters"
C2_COUNT = 1 << 28      # 268,435,456 fp32 = 1 GiB per buffer
C3_BYTES = 4 << 30      # 4 GiB per rank
GIB = float(1 << 30)
XGMI_LINK_GBPS = 76.8  # one xGMI link, one direction: the brief's 153 GB/s per link counts both directions


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline_c2(budget_s: float = 12.0) -> dict:
    """The reference's CPU reduce (AicpuReduceTemplate<float> SUM, one core, -O3 no fast-math; restated in
    oracle/hccl_oracle.c) over the full C2 workload, repeated within a bounded time budget."""
    from oracle import oracle as O  # checker / baseline only

    rng = np.random.default_rng(0x5EED0002)
    src = rng.random(C2_COUNT, dtype=np.float32)
    dst = rng.random(C2_COUNT, dtype=np.float32)
    times = []
    t_end = time.perf_counter() + budget_s
    while len(times) < 3 or (time.perf_counter() < t_end and len(times) < 20):
        t0 = time.perf_counter()
        ret = O.aicpu_reduce(O.FP32, O.SUM, dst, src)
        times.append(time.perf_counter() - t0)
        assert ret == 0
    med = float(np.median(times))
    # the same loop split over the host threads this job may use (labelled separately): slices of
    # the pair, one per thread (the oracle's C call releases the GIL)
    from concurrent.futures import ThreadPoolExecutor

    threads = max(1, min(16, os.cpu_count() or 1))  # the GPU box's CPU share for one GPU is 16
    bounds = np.linspace(0, C2_COUNT, threads + 1).astype(np.int64)
    mt = []
    with ThreadPoolExecutor(threads) as pool:
        for _ in range(5):
            t0 = time.perf_counter()
            rets = list(pool.map(lambda i: O.aicpu_reduce(O.FP32, O.SUM, dst[bounds[i]:bounds[i + 1]],
                                                          src[bounds[i]:bounds[i + 1]]), range(threads)))
            mt.append(time.perf_counter() - t0)
            assert all(r == 0 for r in rets)
    return {
        "value": round(3 * C2_COUNT * 4 / med / GIB, 3),
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"full C2 workload (dst = src + dst over 2 x 1 GiB fp32), {len(times)} passes, median; "
                  f"host {cpu_model()}, nproc {os.cpu_count()}",
        "all_cores": {"value": round(3 * C2_COUNT * 4 / float(np.median(mt)) / GIB, 3), "unit": "GiB/s",
                      "cores": threads, "sample": "same workload split into one slice per thread, 5 passes, median"},
    }


def c1_sim_replay() -> dict:
    """Config C1: 2-rank AllReduce SUM, 1 MiB fp32, the product's schedules replayed on the host by the oracle's
    sim world (the reference's only multi-rank-without-hardware path is its host simulator)."""
    from oracle import oracle as O

    count = (1 << 20) // 4
    progs, scratch = [], 0
    for r in range(2):
        arr, nops, algo, se = H.build_schedule(H.OpType.ALLREDUCE, H.Algo.AUTO, 2, r, count, H.HcclDataType.FP32)
        progs.append((arr, nops))
        scratch = max(scratch, se)
    rng = np.random.default_rng(0x5EED0001)
    xs = [rng.random(count, dtype=np.float32) for _ in range(2)]
    times = []
    for _ in range(7):
        bufs = [[x.copy(), np.zeros(count, np.float32), np.zeros(max(scratch, 1), np.float32)] for x in xs]
        t0 = time.perf_counter()
        assert O.replay(2, O.FP32, O.SUM, progs, bufs) == 0
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    return {"workload": "C1: 2-rank AllReduce SUM 1 MiB fp32, schedule replay on host (one-shot, order O1)",
            "us": round(med * 1e6, 1), "GiBps_per_rank_input": round((1 << 20) / med / GIB, 3), "cores": 1}


def cpu_baseline_allreduce(world: int, algo: int, nbytes: int = 16 << 20, budget_s: float = 10.0) -> dict:
    """The reference's CPU path at N > 1: every rank's program of this N-rank AllReduce (fp32 SUM, `nbytes` per rank,
    the headline's schedule) replayed on the host by the oracle's sim world (AicpuReduceTemplate folds, one FIFO per
    rank pair; one core), timed within a bounded budget. value = whole-job reduced input GiB/s, the unit of the line's
    `value`."""
    from oracle import oracle as O  # checker / baseline only

    count = nbytes // 4
    progs, scratch = [], 0
    for r in range(world):
        arr, nops, _, se = H.build_schedule(H.OpType.ALLREDUCE, algo, world, r, count, H.HcclDataType.FP32)
        progs.append((arr, nops))
        scratch = max(scratch, se)
    rng = np.random.default_rng(0x5EED0004)
    xs = [rng.random(count, dtype=np.float32) for _ in range(world)]
    times = []
    t_end = time.perf_counter() + budget_s
    while len(times) < 2 or (time.perf_counter() < t_end and len(times) < 10):
        bufs = [[x.copy(), np.zeros(count, np.float32), np.zeros(max(scratch, 1), np.float32)] for x in xs]
        t0 = time.perf_counter()
        assert O.replay(world, O.FP32, O.SUM, progs, bufs) == 0
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    return {"value": round(world * nbytes / med / GIB, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{world}-rank AllReduce fp32 SUM, {nbytes >> 20} MiB per rank, {H.Algo(algo).name} schedule: "
                      f"every rank's program replayed on the host by the oracle's sim world, {len(times)} passes, "
                      f"median; host {cpu_model()}"}


def end_to_end_host(steps: int = 5, chunk: int = 64 << 20) -> dict:
    """Gradient buckets that start and end in host memory (BASELINE.json): pinned H2D of both operands, the reduce,
    D2H of the result. Two forms, both reported:
      serial     one stream, whole buffers (H2D 2 GiB, reduce, D2H 1 GiB);
      pipelined  chunks of `chunk` bytes per operand on three streams (H2D / reduce / D2H joined by events), so
                 H2D of chunk i+1, the reduce of chunk i and D2H of chunk i-1 overlap and PCIe runs both directions.
    Rate = 3 GiB of algorithmic bytes per step over the wall time of the step."""
    dev = torch.device("cuda", 0)
    h_src = torch.empty(C2_COUNT, dtype=torch.float32).pin_memory()
    h_dst = torch.empty(C2_COUNT, dtype=torch.float32).pin_memory()
    h_out = torch.empty(C2_COUNT, dtype=torch.float32).pin_memory()
    h_src.uniform_(-1, 1)
    h_dst.uniform_(-1, 1)
    d_src = torch.empty(C2_COUNT, device=dev)
    d_dst = torch.empty(C2_COUNT, device=dev)
    s = torch.cuda.current_stream()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(4)]

    def serial(rec):
        if rec:
            evs[0].record(s)
        d_src.copy_(h_src, non_blocking=True)
        d_dst.copy_(h_dst, non_blocking=True)
        if rec:
            evs[1].record(s)
        H.local_reduce(d_dst, d_src, H.HcclReduceOp.SUM, s)
        if rec:
            evs[2].record(s)
        h_out.copy_(d_dst, non_blocking=True)
        if rec:
            evs[3].record(s)

    serial(False)
    torch.cuda.synchronize()
    parts = []
    t0 = time.perf_counter()
    for _ in range(steps):
        serial(True)
        torch.cuda.synchronize()
        parts.append([evs[i].elapsed_time(evs[i + 1]) for i in range(3)])
    wall = (time.perf_counter() - t0) / steps
    h2d, red, d2h = (float(np.median([p[i] for p in parts])) for i in range(3))
    ok_serial = bool(torch.equal(h_out[:: 1 << 16], (h_src + h_dst)[:: 1 << 16]))

    up, mid, down = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    per = chunk // 4
    nchunks = (C2_COUNT + per - 1) // per

    def pipelined():
        for i in range(nchunks):
            sl = slice(i * per, min(C2_COUNT, (i + 1) * per))
            with torch.cuda.stream(up):
                d_src[sl].copy_(h_src[sl], non_blocking=True)
                d_dst[sl].copy_(h_dst[sl], non_blocking=True)
                e_up = torch.cuda.Event()
                e_up.record(up)
            mid.wait_event(e_up)
            H.local_reduce(d_dst[sl], d_src[sl], H.HcclReduceOp.SUM, mid)
            e_mid = torch.cuda.Event()
            e_mid.record(mid)
            down.wait_event(e_mid)
            with torch.cuda.stream(down):
                h_out[sl].copy_(d_dst[sl], non_blocking=True)
        torch.cuda.synchronize()

    h_out.zero_()
    pipelined()
    ok_pipe = bool(torch.equal(h_out[:: 1 << 16], (h_src + h_dst)[:: 1 << 16]))
    t0 = time.perf_counter()
    for _ in range(steps):
        pipelined()
    wall_p = (time.perf_counter() - t0) / steps
    return {"GiBps": round(3 * C2_COUNT * 4 / wall_p / GIB, 2), "ms_per_step": round(wall_p * 1e3, 2),
            "form": f"pipelined: {chunk >> 20} MiB chunks, H2D / reduce / D2H on three streams",
            "result_ok": ok_pipe,
            "serial": {"GiBps": round(3 * C2_COUNT * 4 / wall / GIB, 2), "ms_per_step": round(wall * 1e3, 2),
                       "h2d_ms": round(h2d, 2), "reduce_ms": round(red, 3), "d2h_ms": round(d2h, 2),
                       "h2d_GBps": round(2 * C2_COUNT * 4 / (h2d / 1e3) / 1e9, 1),
                       "d2h_GBps": round(C2_COUNT * 4 / (d2h / 1e3) / 1e9, 1), "result_ok": ok_serial},
            "note": "pinned host buffers; 2 GiB H2D + reduce + 1 GiB D2H per step (PCIe-bound)"}


def pmc_traffic(name: str):
    """(HBM bytes per launch, provenance) from the newest committed rocprofv3 PMC summary of this kernel
    (profiles/<round>_pmc_<name>.json, tools/profile_round.sh). The counters are never measured inside this run (a
    counter pass is a run of its own under rocprofv3, MI355X_MICROARCH.md), so the line says where they came from and
    whether they were taken on the library it has loaded."""
    import glob
    import hashlib

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_pmc_{name}.json")),
                   key=lambda p: os.path.basename(p).split("_pmc_")[0])
    if not files:
        return None, {"file": None, "measured_in_run": False}
    path = files[-1]
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError) as e:
        return None, {"file": os.path.relpath(path, ROOT), "error": str(e), "measured_in_run": False}
    try:
        with open(H.LIB_PATH, "rb") as f:
            loaded = hashlib.sha256(f.read()).hexdigest()
    except OSError:
        loaded = None
    profiled = d.get("library_sha256")
    return d.get("hbm_bytes_per_launch"), {
        "file": os.path.relpath(path, ROOT),
        "source_commit": d.get("source_commit"),
        "library_sha256": profiled,
        # False: the counters were taken on another build of the library than the one this line measured
        "library_matches": (profiled == loaded) if profiled and loaded else None,
        "traffic_over_algorithmic": d.get("traffic_over_algorithmic"),
        "measured_in_run": False,
    }


def fold_roofline(dev, stream, n: int = 8, reps: int = 10) -> dict:
    """k_reduceN over n fresh 1 GiB fp32 inputs into a 1 GiB output: per-launch duration (HIP events on the launch
    stream), achieved algorithmic GB/s against the HBM peak, the PMC traffic of the committed profile, and the output
    checked bit-exact against the same left fold on torch (acc = x0; acc = x_j + acc)."""
    count = C2_COUNT
    g = torch.Generator(device=dev).manual_seed(0x5EED0008)
    ins = [torch.rand(count, device=dev, generator=g).mul_(2).sub_(1) for _ in range(n)]
    out = torch.empty(count, device=dev)
    H.local_reduce_n(out, ins, H.HcclReduceOp.SUM, stream)
    torch.cuda.synchronize()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    evs[0].record(stream)
    for k in range(reps):
        H.local_reduce_n(out, ins, H.HcclReduceOp.SUM, stream)
        evs[k + 1].record(stream)
    torch.cuda.synchronize()
    per = [evs[k].elapsed_time(evs[k + 1]) / 1e3 for k in range(reps)]
    acc = ins[0].clone()
    for x in ins[1:]:
        acc = torch.add(x, acc)
    ok = bool(torch.equal(out, acc))
    nbytes = (n + 1) * count * 4
    kavg = float(np.mean(per))
    del ins, out, acc
    traffic, source = pmc_traffic("fold_n8")
    return {"kernel": "k_reduceN<EFp<float>, SUM> (8 inputs)", "algorithmic_bytes_per_launch": nbytes,
            "kernel_avg_us": round(kavg * 1e6, 1), "kernel_median_us": round(float(np.median(per)) * 1e6, 1),
            "achieved_GBps": round(nbytes / kavg / 1e9, 1), "peak_GBps": HBM_PEAK_GBPS,
            "frac": round(nbytes / kavg / 1e9 / HBM_PEAK_GBPS, 4),
            "traffic": traffic, "traffic_source": source,
            "result_ok": ok}


def ipc_two_shot_roofline(dev, n: int = 2, mib: int = 512, reps: int = 10) -> dict:
    """The one-sided kernel (k_ipc_collective, the AIV engine's analogue) on one GPU: an n-rank
    loopback world (every rank's blocks in one launch on rank 0's stream, each rank driven from its own host thread),
    two-shot AllReduce fp32 SUM of `mib` MiB per rank. Per rank and launch the kernel reads and writes
    2(3n-2)/n bytes per input byte (phase 0 stores (n-1)/n of the input into the owners' slots, phase 1 folds the own
    chunk and n-1 slots and writes n results, phase 2 copies n-1 results), all of it this GPU's HBM here. Checked
    against torch's add in the two-shot order O2 (acc = x0; acc = x1 + acc)."""
    from concurrent.futures import ThreadPoolExecutor

    # phase stamps on (read at the world's IPC set-up): each launch's own span, first block in to last block out, is
    # the kernel's duration; the HIP events between calls also hold the loopback world's cross-stream hand-offs
    prev = {k: os.environ.get(k) for k in ("HCCL_AMD_IPC_TRACE", "HCCL_BUFFSIZE", "HCCL_AMD_IPC_STAGING_MIB")}
    os.environ["HCCL_AMD_IPC_TRACE"] = "1"
    # the large staging tier's areas are HCCL_BUFFSIZE / 2 (the reference's 2 x HCCL_BUFFSIZE for the four): a caller
    # that moves 512 MiB per call sets HCCL_BUFFSIZE to 1024, as on the reference, and each call is one staging round
    # (the rows before r06 ran with 512 MiB areas, the default then)
    os.environ["HCCL_BUFFSIZE"] = "1024"
    os.environ.pop("HCCL_AMD_IPC_STAGING_MIB", None)
    comms = H.loopback_world(n)
    count = (mib << 20) // 4
    g = torch.Generator(device=dev).manual_seed(0x5EED0009)
    xs = [torch.rand(count, device=dev, generator=g).mul_(2).sub_(1) for _ in range(n)]
    ys = [torch.empty_like(x) for x in xs]
    streams = [torch.cuda.Stream() for _ in range(n)]
    torch.cuda.synchronize()
    pool = ThreadPoolExecutor(n)
    try:
        for c in comms:
            c.set_algo(H.Algo.IPC_TWOSHOT)

        def call():
            list(pool.map(lambda r: comms[r].all_reduce(xs[r], ys[r], H.HcclReduceOp.SUM, streams[r]), range(n)))

        call()  # set-up (staging, peer pointers) on the first call
        torch.cuda.synchronize()
        for k, v in prev.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
        evs[0].record(streams[0])
        for k in range(reps):
            call()
            evs[k + 1].record(streams[0])  # the world's launch runs on rank 0's stream
        torch.cuda.synchronize()
        per_call = [evs[k].elapsed_time(evs[k + 1]) / 1e3 for k in range(reps)]
        per = []
        for _ in range(reps):
            call()
            torch.cuda.synchronize()
            st, blocks = comms[0].ipc_trace()
            a = st[:n, :blocks, :].astype(np.int64)
            per.append(float(a[:, :, 7].max() - a[:, :, 0].min()) * 1e-8)  # s_memrealtime: 100 MHz
        want = torch.add(xs[1], xs[0]) if n == 2 else None
        ok = want is not None and all(bool(torch.equal(y, want)) for y in ys)
        ran = H.Algo(comms[0].last_algo).name
        timeouts = comms[0].ipc_status() & 1
    finally:
        pool.shutdown()
        for c in comms:
            c.destroy()
    nbytes = n * 2 * (3 * n - 2) * count * 4 // n
    kavg = float(np.mean(per))
    traffic, source = pmc_traffic("ipc_two_shot")
    return {"kernel": "k_ipc_collective<EFp<float>, SUM> (two-shot AllReduce, loopback world)", "ranks": n,
            "bytes_per_rank": count * 4, "ran": ran, "algorithmic_bytes_per_launch": nbytes,
            "staging": "HCCL_BUFFSIZE=1024: large-tier areas of 512 MiB, one staging round per call",
            "kernel_avg_us": round(kavg * 1e6, 1), "kernel_median_us": round(float(np.median(per)) * 1e6, 1),
            "kernel_timing": "each launch's span from its blocks' s_memrealtime stamps (first entry to last exit; "
                             "HCCL_AMD_IPC_TRACE), one launch per call",
            "call_to_call_avg_us": round(float(np.mean(per_call)) * 1e6, 1),
            "achieved_GBps": round(nbytes / kavg / 1e9, 1), "peak_GBps": HBM_PEAK_GBPS,
            "frac": round(nbytes / kavg / 1e9 / HBM_PEAK_GBPS, 4),
            "traffic": traffic, "traffic_source": source,
            "barrier_timeouts": timeouts,
            "result_ok": ok}


def _device_memory_outside_torch() -> int:
    """Bytes in use on the current device that torch's caching allocator does not hold (hipMemGetInfo minus torch's
    reserved bytes): RCCL's and this library's device allocations, plus the runtime's own."""
    free, total = torch.cuda.mem_get_info()
    return int(total - free - torch.cuda.memory_reserved())


def fold_piece_loopback(n: int = 8, mib: int = 256) -> dict:
    """The fold at its operating point inside a program on one GPU: the reference's C3
    selection (MeshChunk, O6) on an n-rank loopback world, `mib` MiB fp32 per rank, every fold launch of rank 0's
    program timed on its reduce stream (Config.FOLD_TIMING). The folds read MeshChunk sub-slices that the world's links
    (the library's copy kernel) have just written, so this is the fold on fresh staging at the schedule's piece sizes;
    the span is the loopback harness's, not xGMI's (its host rendezvous per group). All n ranks' programs run on this
    one GPU at once, so the fold figures are rank 0's share under contention (r05: 998 GB/s per fold with 8 ranks, about
    1/8 of HBM); they show the program's fold count and piece sizes, not the kernel's speed. The N > 1 line's
    fold_piece row is the same measurement over RCCL on xGMI, one rank per GPU."""
    from concurrent.futures import ThreadPoolExecutor

    comms = H.loopback_world(n)
    count = (mib << 20) // 4
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0x5EED000A)
    xs = [torch.rand(count, device=dev, generator=g) for _ in range(n)]
    ys = [torch.empty_like(x) for x in xs]
    streams = [torch.cuda.Stream() for _ in range(n)]
    pool = ThreadPoolExecutor(n)
    try:
        for c in comms:
            c.set_algo(H.Algo.MESH_CHUNK)
            c.set_config(H.Config.FOLD_TIMING, 1)
        torch.cuda.synchronize()
        rows = []
        for _ in range(3):
            list(pool.map(lambda r: comms[r].all_reduce(xs[r], ys[r], H.HcclReduceOp.SUM, streams[r]), range(n)))
            torch.cuda.synchronize()
            rows.append(comms[0].fold_timing())
        t = rows[-1]
        ran = H.Algo(comms[0].last_algo).name
    finally:
        pool.shutdown()
        torch.cuda.synchronize()
        for c in comms:
            c.destroy()
    fold_us = float(np.median([r["fold_us"] for r in rows[1:]]))
    return {"workload": f"C3 selection (MeshChunk) on a {n}-rank loopback world, {mib} MiB fp32 per rank; rank 0's folds",
            "ran": ran, "folds": t["folds"], "fold_bytes": t["fold_bytes"],
            "bytes_per_fold": t["fold_bytes"] // max(1, t["folds"]), "fold_us": round(fold_us, 1),
            "fold_avg_us": round(fold_us / max(1, t["folds"]), 2),
            "fold_GBps": round(t["fold_bytes"] / (fold_us * 1e-6) / 1e9, 1),
            "fold_frac_hbm": round(t["fold_bytes"] / (fold_us * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4),
            "span_us": round(t["span_us"], 1),
            "concurrent_ranks": n,
            "note": "fold durations are HIP-event brackets of each fold launch on the reduce stream (median of the last "
                    "two of three calls). All ranks share this GPU, so each fold runs beside the other ranks' folds and "
                    "link copies: fold_GBps is rank 0's share of HBM under that contention, not the fold kernel's rate "
                    "(C2 and fold_n8 are), and the span is harness-bound. The N > 1 line's fold_piece row is the "
                    "uncontended operating point"}


def bench_local(args) -> dict:
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0x5EED0002)
    src = torch.rand(C2_COUNT, device=dev, generator=g).mul_(2).sub_(1)
    dst = torch.rand(C2_COUNT, device=dev, generator=g).mul_(2).sub_(1)
    stream = torch.cuda.current_stream()
    for _ in range(args.warmup):
        H.local_reduce(dst, src, H.HcclReduceOp.SUM, stream)
    torch.cuda.synchronize()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    evs[0].record(stream)
    for k in range(args.steps):
        H.local_reduce(dst, src, H.HcclReduceOp.SUM, stream)
        evs[k + 1].record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    per = [evs[k].elapsed_time(evs[k + 1]) / 1e3 for k in range(args.steps)]
    # the measured kernel on the measured buffers, once more after the timed region: dst' = src + dst must be the
    # IEEE sum torch computes elementwise (same bits: one correctly rounded add per element)
    before = dst.clone()
    H.local_reduce(dst, src, H.HcclReduceOp.SUM, stream)
    torch.cuda.synchronize()
    result_ok = bool(torch.equal(dst, torch.add(src, before)))
    del before
    total = evs[0].elapsed_time(evs[-1]) / 1e3
    bytes_step = 3 * C2_COUNT * 4
    value = bytes_step * args.steps / total / GIB
    kavg = float(np.mean(per))
    achieved = bytes_step / kavg / 1e9
    traffic, traffic_source = pmc_traffic("local_reduce")
    log(f"[bench] C2 local reduce: {value:.1f} GiB/s  kernel avg {kavg*1e6:.1f} us  min {min(per)*1e6:.1f} us  "
        f"max {max(per)*1e6:.1f} us  host wall {wall:.3f} s")
    res = {
        "metric": "device-resident reduce GiB/s (fp32 sum) vs HBM peak; ring all-reduce bus GB/s",
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(total / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (uniform [-1,1) fp32, device-generated)",
        "result_ok": result_ok,
        "config": {
            "workload": "C2: 1-GPU local reduce dst = src + dst (HcclAmdLocalReduce), 2 x 1 GiB fp32 in HBM",
            "count": C2_COUNT,
            "bytes_per_step": bytes_step,
            "parallelism": "single GPU",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": traffic,
            "traffic_source": traffic_source,
            "kernel": "k_reduce2<EFp<float>, SUM>",
            "algorithmic_bytes_per_launch": bytes_step,
            "kernel_avg_us": round(kavg * 1e6, 2),
            "kernel_median_us": round(float(np.median(per)) * 1e6, 2),
            "kernel_p10_us": round(float(np.percentile(per, 10)) * 1e6, 2),
            "kernel_p90_us": round(float(np.percentile(per, 90)) * 1e6, 2),
        },
        # the same quantities at every N: buffer bytes per GPU per second (algbw), the bytes the
        # bounding resource moves per second (busbw: HBM here, xGMI at N > 1) and its fraction of that roofline
        "per_gpu": {"workload": "C2", "bytes_per_gpu_per_step": C2_COUNT * 4,
                    "algbw_GBps": round(C2_COUNT * 4 / (total / args.steps) / 1e9, 2),
                    "busbw_GBps": round(bytes_step / (total / args.steps) / 1e9, 2), "bound": "hbm",
                    "roofline_peak_GBps": HBM_PEAK_GBPS,
                    "frac": round(bytes_step / (total / args.steps) / 1e9 / HBM_PEAK_GBPS, 4)},
    }
    # the same stream shapes on PyTorch's own kernels, same buffers and stream: the vendor-library baseline for this
    # op (torch.add, 2 reads + 1 write) and the 1 read + 1 write copy, as measured context for `frac`
    try:
        out = torch.empty_like(dst)

        def rate(fn, nbytes, reps=10):
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                fn()
            e1.record(stream)
            torch.cuda.synchronize()
            return round(nbytes / (e0.elapsed_time(e1) / 1e3 / reps) / 1e9, 1)

        res["roofline"]["same_op_on_torch"] = {
            "torch_add_GBps": rate(lambda: torch.add(src, dst, out=out), bytes_step),
            "torch_copy_GBps": rate(lambda: out.copy_(src), 2 * C2_COUNT * 4),
            "note": "torch.add(src, dst, out) over the same 2 x 1 GiB fp32 (3 GiB per call) and a 1 GiB copy",
        }
        del out
    except Exception as e:  # noqa: BLE001
        res["roofline"]["same_op_on_torch"] = {"error": f"{type(e).__name__}: {e}"}
    # The kernel VERDICT r01 named furthest below its roofline: the ordered 8-input fold that the mesh schedules run
    # at C3 (k_reduceN, 8 x 1 GiB fp32 in, 1 GiB out; (n+1) x 1 GiB algorithmic bytes per launch). Context beside the
    # headline, never `value`; its placement spread is in DESIGN.md §3.
    try:
        res["other_kernels"] = {"fold_n8": fold_roofline(dev, stream)}
    except Exception as e:  # noqa: BLE001
        res["other_kernels"] = {"fold_n8": {"error": f"{type(e).__name__}: {e}"}}
    try:
        res["other_kernels"]["ipc_two_shot"] = ipc_two_shot_roofline(dev)
    except Exception as e:  # noqa: BLE001
        res["other_kernels"]["ipc_two_shot"] = {"error": f"{type(e).__name__}: {e}"}
    try:
        res["other_kernels"]["fold_piece_loopback"] = fold_piece_loopback()
    except Exception as e:  # noqa: BLE001
        res["other_kernels"]["fold_piece_loopback"] = {"error": f"{type(e).__name__}: {e}"}
    if not args.no_e2e:
        try:
            res["end_to_end_host_buffers"] = end_to_end_host()
        except Exception as e:  # noqa: BLE001  (reported, never fatal to the headline line)
            res["end_to_end_host_buffers"] = {"error": f"{type(e).__name__}: {e}"}
    if not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline_c2(args.cpu_budget)
        res["cpu_baseline"]["c1_sim"] = c1_sim_replay()
    return res


def rccl_allreduce_reference(send, recv, world, args):
    """RCCL's own ring/tree all_reduce on the same 4 GiB buffers (torch.distributed nccl backend = RCCL), for
    context only: it is the vendor baseline the schedules here are compared against."""
    import torch.distributed as dist

    try:
        g = dist.new_group(backend="nccl")
        recv.copy_(send)
        f = (world - 1) / world
        n = max(3, args.steps // 2)
        t = _timed(lambda: dist.all_reduce(recv, group=g), n)
        out = {"ms_per_step": round(t * 1e3, 3), "busbw_GBps": round(C3_BYTES / t / 1e9 * 2 * f, 2)}
        # The two data movements of the two-shot on RCCL's own kernels, same bytes per rank: the all-to-all that
        # the scatter phase is (every rank sends 1/n of its buffer to each peer) and the ring all-gather of the
        # gather phase. They bound what p2p groups over the same links can reach.
        t = _timed(lambda: dist.all_to_all_single(recv, send, group=g), 3)
        out["alltoall_ms"] = round(t * 1e3, 3)
        out["alltoall_busbw_GBps"] = round(C3_BYTES / t / 1e9 * f, 2)
        shard = send[: send.numel() // world]
        t = _timed(lambda: dist.all_gather_into_tensor(recv, shard, group=g), 3)
        out["allgather_ms"] = round(t * 1e3, 3)
        out["allgather_busbw_GBps"] = round(C3_BYTES / t / 1e9 * f, 2)
        # B_link: RCCL send/recv of 1 GiB between ranks 0 and 1 over their one direct link, one way
        # and both ways at once; the other ranks only take part in the barriers
        rank = dist.get_rank()
        nbytes = 1 << 30
        a, b = send.view(torch.uint8)[:nbytes], recv.view(torch.uint8)[:nbytes]

        def p2p(both):
            ops = []
            if rank == 0:
                ops.append(dist.P2POp(dist.isend, a, 1, g))
                if both:
                    ops.append(dist.P2POp(dist.irecv, b, 1, g))
            elif rank == 1:
                ops.append(dist.P2POp(dist.irecv, b, 0, g))
                if both:
                    ops.append(dist.P2POp(dist.isend, a, 0, g))
            for req in dist.batch_isend_irecv(ops) if ops else ():
                req.wait()

        if dist.get_world_size() < 2:
            out["link_probe"] = {"skipped": "one rank (the self-loop stand-in): no link to probe"}
            return out
        try:
            t = _timed(lambda: p2p(False), 3)
            out["link_probe"] = {"pair": [0, 1], "bytes": nbytes, "one_way_GBps": round(nbytes / t / 1e9, 2)}
            t = _timed(lambda: p2p(True), 3)
            out["link_probe"]["both_ways_GBps_per_direction"] = round(nbytes / t / 1e9, 2)
        except Exception as e:  # noqa: BLE001  (the probe never hides the rows above)
            out["link_probe"] = {"error": f"{type(e).__name__}: {e}"}
        return out
    except Exception as e:  # noqa: BLE001
        return {"error": f"{type(e).__name__}: {e}"}


def _timed(fn, iters: int, warmup: int = 2) -> float:
    """Per-iteration seconds of fn() on the current stream, max over ranks (barrier before and after)."""
    import torch.distributed as dist

    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    dist.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    dist.barrier()
    t = torch.tensor([e0.elapsed_time(e1) / 1e3 / iters], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0])


def _graph_us(call, calls: int = 50, replays: int = 5) -> float:
    """Per-call microseconds of `call(stream)` captured `calls` times in one HIP graph and replayed, max over ranks.
    Every rank captures the same calls, so the replays' barriers pair up."""
    import torch.distributed as dist

    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=torch.cuda.Stream()):
        st = torch.cuda.current_stream()
        for _ in range(calls):
            call(st)
    g.replay()
    torch.cuda.synchronize()
    dist.barrier()
    cur = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(cur)
    for _ in range(replays):
        g.replay()
    e1.record(cur)
    torch.cuda.synchronize()
    dist.barrier()
    t = torch.tensor([e0.elapsed_time(e1) * 1e3 / (calls * replays)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    del g
    return float(t[0])


def _xgmi_frac(busbw_GBps: float, world: int):
    """busbw as a fraction of the xGMI algorithmic-bus roofline a rank has (one 76.8 GB/s link per peer, at most 7);
    None in the one-GPU harness and self-loop modes, which have no xGMI in the path."""
    if os.environ.get("HCCL_AMD_BENCH_HOST_EXCHANGE") == "1" or os.environ.get("HCCL_AMD_BENCH_SELFLOOP") == "1" \
            or world < 2:
        return None
    return round(busbw_GBps / (min(world - 1, 7) * XGMI_LINK_GBPS), 4)


def bench_c4(comm, send, recv, world) -> dict:
    """C4: ZeRO-style gradient bucket, bf16, 2 GiB per rank: HcclReduceScatter (SUM) then HcclAllGather."""
    nbytes = 2 << 30
    x = send.view(torch.bfloat16)[: nbytes // 2]
    full = recv.view(torch.bfloat16)[: nbytes // 2]
    shard = torch.empty(x.numel() // world, dtype=torch.bfloat16, device=x.device)
    s = torch.cuda.current_stream()
    t_rs = _timed(lambda: comm.reduce_scatter(x, shard, H.HcclReduceOp.SUM, s), 5)
    rs_algo = H.Algo(comm.last_algo).name  # MESH_CHUNK at this size, as the reference selects
    t_ag = _timed(lambda: comm.all_gather(shard, full, s), 5)
    f = (world - 1) / world
    out = {"workload": "C4: ReduceScatter + AllGather bf16 SUM, 2 GiB per rank", "rs_algo": rs_algo,
           "rs_ms": round(t_rs * 1e3, 3), "ag_ms": round(t_ag * 1e3, 3),
           "rs_busbw_GBps": round(nbytes / t_rs / 1e9 * f, 2), "ag_busbw_GBps": round(nbytes / t_ag / 1e9 * f, 2),
           "rs_ag_busbw_GBps": round(2 * nbytes / (t_rs + t_ag) / 1e9 * f, 2)}
    out["rs_ag_xgmi_frac"] = _xgmi_frac(out["rs_ag_busbw_GBps"], world)
    # the mesh ReduceScatter (order O1) and the one-sided IPC kernel with the same order: same bits; then the IPC
    # kernel in the auto family (MeshChunk O6 here), which must match the auto ReduceScatter
    try:
        comm.set_algo(H.Algo.MESH_ONESHOT)
        t_mesh = _timed(lambda: comm.reduce_scatter(x, shard, H.HcclReduceOp.SUM, s), 3, warmup=1)
        out["rs_mesh_ms"] = round(t_mesh * 1e3, 3)
        mesh_ran = H.Algo(comm.last_algo).name
        ref = shard.view(torch.int16)[:: 1 << 10].clone()
        comm.set_algo(H.Algo.IPC_TWOSHOT)
        t_ipc = _timed(lambda: comm.reduce_scatter(x, shard, H.HcclReduceOp.SUM, s), 5)
        out["rs_ipc_ms"] = round(t_ipc * 1e3, 3)
        out["rs_ipc_busbw_GBps"] = round(nbytes / t_ipc / 1e9 * f, 2)
        out["rs_ipc_xgmi_frac"] = _xgmi_frac(out["rs_ipc_busbw_GBps"], world)
        out["rs_ipc_ran"] = H.Algo(comm.last_algo).name
        # only when the mesh row ran its own schedule (order O1; the one-GPU harness runs the auto family there)
        out["rs_ipc_matches_mesh"] = (bool(torch.equal(ref, shard.view(torch.int16)[:: 1 << 10]))
                                      if mesh_ran == "MESH_ONESHOT" else None)
        out["rs_mesh_ran"] = mesh_ran
        out["rs_ipc_barrier_timeouts"] = comm.ipc_status() & 1
        comm.set_algo(H.Algo.AUTO)
        comm.reduce_scatter(x, shard, H.HcclReduceOp.SUM, s)
        ref_auto = shard.view(torch.int16)[:: 1 << 10].clone()
        comm.set_algo(H.Algo.IPC)
        t_ipc9 = _timed(lambda: comm.reduce_scatter(x, shard, H.HcclReduceOp.SUM, s), 5)
        out["rs_ipc_auto_family_ms"] = round(t_ipc9 * 1e3, 3)
        out["rs_ipc_auto_family_busbw_GBps"] = round(nbytes / t_ipc9 / 1e9 * f, 2)
        out["rs_ipc_auto_family_ran"] = H.Algo(comm.last_algo).name
        out["rs_ipc_auto_family_matches_auto"] = bool(torch.equal(ref_auto, shard.view(torch.int16)[:: 1 << 10]))
    except H.HcclError as e:
        out["rs_rows_error"] = str(e)
    finally:
        comm.set_algo(H.Algo.AUTO)
    # the AllGather half on the IPC kernel (one launch per call, data movement only) beside the RCCL mesh above
    try:
        comm.set_algo(H.Algo.AUTO)
        comm.all_gather(shard, full, s)
        ref_ag = full.view(torch.int16)[:: 1 << 10].clone()
        comm.set_algo(H.Algo.IPC)
        t_ag_ipc = _timed(lambda: comm.all_gather(shard, full, s), 5)
        out["ag_ipc_ms"] = round(t_ag_ipc * 1e3, 3)
        out["ag_ipc_busbw_GBps"] = round(nbytes / t_ag_ipc / 1e9 * f, 2)
        out["ag_ipc_xgmi_frac"] = _xgmi_frac(out["ag_ipc_busbw_GBps"], world)
        out["ag_ipc_ran"] = H.Algo(comm.last_algo).name
        out["ag_ipc_matches_auto"] = bool(torch.equal(ref_ag, full.view(torch.int16)[:: 1 << 10]))
        out["ag_ipc_barrier_timeouts"] = comm.ipc_status() & 1
    except H.HcclError as e:
        out["ag_ipc_error"] = str(e)
    finally:
        comm.set_algo(H.Algo.AUTO)
    return out


def bench_c5(comm, send, recv, world, max_bytes: int = 4 << 30) -> dict:
    """C5: AllReduce fp16 SUM, 1 KiB .. 4 GiB: latency at small sizes, busbw at large. Rows per size (`<row>_ran` names
    the path that ran, `<row>_us` and `<row>_busbw_GBps` its time):
      rhd / auto        the RHD schedule (the config's algorithm) and the auto selection (what the reference would
                        run), every size, over the transport with the small-call rule off (Config.SMALL_IPC_BYTES 0);
      rhd_default / auto_default   the same calls as a caller gets them by default up to the rule's threshold
                        (1 MiB): one launch of the one-sided kernel in the same order (IPC_RHD / IPC), compared bit for
                        bit with the rhd / auto rows, and from a HIP graph (`*_graph_us`);
      ipc / ipc_rhd     the one-sided kernel forced, up to 256 / 64 MiB.
    The transport rows of every size run before the one-sided ones: an IPC barrier timeout fails the communicator."""
    s = torch.cuda.current_stream()
    sizes = []
    nbytes = 1 << 10
    while nbytes <= max_bytes:
        sizes.append(nbytes)
        nbytes *= 2
    rows = {b: {"bytes": b} for b in sizes}
    f = 2 * (world - 1) / world
    small = comm.get_config(H.Config.SMALL_IPC_BYTES)  # the default threshold (HCCL_AMD_SMALL_IPC_BYTES)
    plan = (("rhd", H.Algo.RHD, 0, max_bytes), ("auto", H.Algo.AUTO, 0, max_bytes),
            ("rhd_default", H.Algo.RHD, small, small), ("auto_default", H.Algo.AUTO, small, small),
            ("ipc", H.Algo.IPC, 0, 256 << 20), ("ipc_rhd", H.Algo.IPC_RHD, 0, 64 << 20))
    twin = {"rhd_default": "rhd", "auto_default": "auto", "ipc_rhd": "rhd", "ipc": "auto"}
    own = {"rhd": "RHD"}  # the path a transport row must have run for a comparison with it to mean anything
    digests = {}
    try:
        for key, algo, rule, limit in plan:
            comm.set_algo(algo)
            comm.set_config(H.Config.SMALL_IPC_BYTES, rule)
            for nbytes in sizes:
                if nbytes > limit:
                    break
                row = rows[nbytes]
                a = send.view(torch.float16)[: nbytes // 2]
                b = recv.view(torch.float16)[: nbytes // 2]
                iters = 20 if nbytes <= (64 << 20) else 3
                ll0 = comm.ipc_ll_launches()
                try:
                    t = _timed(lambda: comm.all_reduce(a, b, H.HcclReduceOp.SUM, s), iters)
                except H.HcclError as e:
                    row[f"{key}_error"] = str(e)
                    continue
                row[f"{key}_us"] = round(t * 1e6, 1)
                row[f"{key}_busbw_GBps"] = round(nbytes / t / 1e9 * f, 2)
                ran = H.Algo(comm.last_algo).name
                row[f"{key}_ran"] = ran
                if nbytes >= (256 << 20):  # the bandwidth end of the curve
                    row[f"{key}_xgmi_frac"] = _xgmi_frac(row[f"{key}_busbw_GBps"], world)
                sample = b.view(torch.int16)[:: 1 << 10].clone()
                digests[(key, nbytes)] = sample
                tw = twin.get(key)
                if tw is not None and (tw, nbytes) in digests:
                    tw_ran = row.get(f"{tw}_ran")
                    # compared only when the twin ran its own schedule (the one-GPU harness runs every row on the
                    # one-sided kernel; the auto twin's family is whatever the selector picked, so any transport path)
                    meaningful = tw_ran == own[tw] if tw in own else (tw_ran is not None and not tw_ran.startswith("IPC"))
                    row[f"{key}_matches_{tw}"] = bool(torch.equal(sample, digests[(tw, nbytes)])) if meaningful else None
                if ran.startswith("IPC"):
                    row[f"{key}_barrier_timeouts"] = comm.ipc_status() & 1
                    row[f"{key}_ll"] = comm.ipc_ll_launches() != ll0  # the LL form ran (HCCL_AMD_IPC_LL_BYTES)
        for nbytes in sizes:
            row = rows[nbytes]
            for key, algo, rule in (("ipc", H.Algo.IPC, 0), ("rhd_default", H.Algo.RHD, small)):
                if nbytes > (1 << 20) or not str(row.get(f"{key}_ran", "")).startswith("IPC"):
                    continue
                # the latency end replayed from a HIP graph (50 captured calls per replay; device-side epochs)
                a = send.view(torch.float16)[: nbytes // 2]
                b = recv.view(torch.float16)[: nbytes // 2]
                try:
                    comm.set_algo(algo)
                    comm.set_config(H.Config.SMALL_IPC_BYTES, rule)
                    row[f"{key}_graph_us"] = round(_graph_us(lambda st: comm.all_reduce(a, b, H.HcclReduceOp.SUM, st)),
                                                   1)
                    row[f"{key}_graph_barrier_timeouts"] = comm.ipc_status() & 1
                except Exception as e:  # noqa: BLE001  (capture problems never end the sweep)
                    row[f"{key}_graph_error"] = f"{type(e).__name__}: {e}"
    finally:
        comm.set_algo(H.Algo.AUTO)
        comm.set_config(H.Config.SMALL_IPC_BYTES, small)
    return {"workload": "C5: AllReduce fp16 SUM, size sweep (RHD schedule and auto selection)",
            "small_call_rule_bytes": small, "points": [rows[b] for b in sizes]}


def bench_fold_piece(comm, send, recv, world) -> dict:
    """The fold kernel at its real operating point: inside the C3 program with the reference's own
    selection (MeshChunk, 4 GiB fp32: batched 8-input folds of the MeshChunk sub-slices over staging a transport group
    has just written) and inside the C4 ReduceScatter (MeshChunk, 2 GiB bf16), every fold launch timed with HIP events
    on the reduce stream (Config.FOLD_TIMING: the calls run eagerly) against the program's span on the caller's stream.
    fold_GBps = the folds' algorithmic bytes ((operands + 1) x elements x size) over their summed durations; whether the
    folds are on the critical path shows in fold_busy_over_span. Max over ranks."""
    import torch.distributed as dist

    s = torch.cuda.current_stream()
    x = send.view(torch.bfloat16)[: (2 << 30) // 2]
    shard = torch.empty(x.numel() // world, dtype=torch.bfloat16, device=x.device)
    out = {"note": "per rank: the second of two calls, eager; fold durations are HIP-event brackets of each fold launch"}
    comm.set_config(H.Config.FOLD_TIMING, 1)
    try:
        for name, algo, call in (
                ("c3_mesh_chunk", H.Algo.MESH_CHUNK, lambda: comm.all_reduce(send, recv, H.HcclReduceOp.SUM, s)),
                ("c3_ring", H.Algo.RING, lambda: comm.all_reduce(send, recv, H.HcclReduceOp.SUM, s)),
                ("c4_rs_mesh_chunk", H.Algo.MESH_CHUNK, lambda: comm.reduce_scatter(x, shard, H.HcclReduceOp.SUM, s))):
            comm.set_algo(algo)
            try:
                call()
                torch.cuda.synchronize()
                dist.barrier()
                call()
                t = comm.fold_timing()
            except H.HcclError as e:
                out[name] = {"error": str(e), "ran": H.Algo(comm.last_algo).name}
                continue
            v = torch.tensor([t["fold_us"], t["span_us"]], dtype=torch.float64)
            dist.all_reduce(v, op=dist.ReduceOp.MAX)
            fold_us, span_us = float(v[0]), float(v[1])
            out[name] = {"ran": H.Algo(comm.last_algo).name, "folds": t["folds"], "fold_bytes": t["fold_bytes"],
                         "bytes_per_fold": t["fold_bytes"] // max(1, t["folds"]),
                         "fold_us": round(fold_us, 1), "fold_avg_us": round(fold_us / max(1, t["folds"]), 2),
                         "fold_GBps": round(t["fold_bytes"] / (fold_us * 1e-6) / 1e9, 1) if fold_us else None,
                         "fold_frac_hbm": round(t["fold_bytes"] / (fold_us * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4)
                         if fold_us else None,
                         "span_us": round(span_us, 1), "fold_busy_over_span": round(fold_us / span_us, 4)
                         if span_us else None}
    finally:
        comm.set_config(H.Config.FOLD_TIMING, 0)
        comm.set_algo(H.Algo.AUTO)
    return out


def recommend_data_paths(c3: dict, c5: dict) -> dict:
    """Which data path each size range should default to, from the rows of one N > 1 line: the
    two paths give the same bits within an order family, so the choice is free for parity. At C3's 4 GiB: the RCCL
    schedule of each order family against its one-sided twin (MESH_CHUNK vs IPC, MESH_TWOSHOT vs IPC_TWOSHOT). Over
    C5's sweep: per size, the faster of the auto schedule over RCCL (`auto`) and the one-sided kernel (`auto_default`
    up to the small-call threshold, `ipc` above it), then maximal runs of sizes with the same winner. Rows that errored,
    or whose path did not run what it names, are left out."""
    out = {"c3": {}, "c5_ranges": [], "note": "faster path per order family / size range; same bits either way"}
    for rccl, ipc in (("MESH_CHUNK", "IPC"), ("MESH_TWOSHOT", "IPC_TWOSHOT")):
        a, b = (c3 or {}).get(rccl, {}), (c3 or {}).get(ipc, {})
        if "ms" in a and "ms" in b and a.get("ran") == rccl and str(b.get("ran", "")).startswith("IPC"):
            out["c3"][rccl.lower()] = {"rccl_ms": a["ms"], "one_sided_ms": b["ms"],
                                       "choose": "one_sided" if b["ms"] < a["ms"] else "rccl"}
    runs = []
    for row in (c5 or {}).get("points", []):
        rccl_us = row.get("auto_us") if not str(row.get("auto_ran", "IPC")).startswith("IPC") else None
        ipc_us = None
        for key in ("auto_default", "ipc"):
            if str(row.get(f"{key}_ran", "")).startswith("IPC") and f"{key}_us" in row:
                ipc_us = row[f"{key}_us"] if ipc_us is None else min(ipc_us, row[f"{key}_us"])
        if rccl_us is None or ipc_us is None:
            continue
        choose = "one_sided" if ipc_us < rccl_us else "rccl"
        if runs and runs[-1]["choose"] == choose:
            runs[-1]["to_bytes"] = row["bytes"]
        else:
            runs.append({"from_bytes": row["bytes"], "to_bytes": row["bytes"], "choose": choose})
    out["c5_ranges"] = runs
    return out


def bench_e2e_allreduce(comm, world, nbytes: int = 256 << 20, iters: int = 5, chunk: int = 32 << 20) -> dict:
    """Gradient bucket that starts and ends in host memory (BASELINE.json): pinned H2D, HcclAllReduce fp32 SUM, D2H,
    nbytes per rank. serial = one stream, whole bucket; pipelined = chunks on three streams (H2D / AllReduce / D2H
    joined by events). Rate = bucket bytes per rank / max-over-ranks time per step."""
    import torch.distributed as dist

    dev = torch.device("cuda", torch.cuda.current_device())
    h = torch.empty(nbytes // 4, dtype=torch.float32).pin_memory()
    h.uniform_(-1, 1)
    d = torch.empty(nbytes // 4, device=dev)
    s = torch.cuda.current_stream()
    up, mid, down = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    per = chunk // 4

    def serial():
        d.copy_(h, non_blocking=True)
        comm.all_reduce(d, d, H.HcclReduceOp.SUM, s)
        h.copy_(d, non_blocking=True)

    def pipelined():
        for i in range(0, d.numel(), per):
            sl = slice(i, min(d.numel(), i + per))
            with torch.cuda.stream(up):
                d[sl].copy_(h[sl], non_blocking=True)
                e_up = torch.cuda.Event()
                e_up.record(up)
            mid.wait_event(e_up)
            comm.all_reduce(d[sl], d[sl], H.HcclReduceOp.SUM, mid)
            e_mid = torch.cuda.Event()
            e_mid.record(mid)
            down.wait_event(e_mid)
            with torch.cuda.stream(down):
                h[sl].copy_(d[sl], non_blocking=True)
        torch.cuda.synchronize()

    out = {"bytes_per_rank": nbytes,
           "note": "pinned host bucket -> H2D -> in-place HcclAllReduce -> D2H (PCIe-bound)"}
    for name, fn in (("serial", serial), ("pipelined", pipelined)):
        fn()
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        t = torch.tensor([(time.perf_counter() - t0) / iters], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        per_step = float(t[0])
        out[name] = {"ms_per_step": round(per_step * 1e3, 3), "GiBps_per_rank": round(nbytes / per_step / GIB, 2),
                     "algo": H.Algo(comm.last_algo).name}
    out["pipelined"]["chunk_bytes"] = chunk
    return out


def bench_c3_algos(comm, send, recv, world) -> dict:
    """C3 shape (fp32 SUM, 4 GiB per rank) under every AllReduce schedule, 3 timed iterations each. Pairs that compute
    the same order are compared bit for bit on a sample of the output: IPC_TWOSHOT vs MESH_TWOSHOT (O2) and IPC (the
    auto family over the one-sided kernel) vs MESH_CHUNK (O6, the auto choice at this size)."""
    import torch.distributed as dist

    s = torch.cuda.current_stream()
    out = {}
    digests = {}
    twin = {H.Algo.IPC_TWOSHOT: H.Algo.MESH_TWOSHOT, H.Algo.IPC: H.Algo.MESH_CHUNK}
    try:
        # (schedule, IPC workgroups per launch; 0 = the default by size). The RCCL schedules run first: an IPC
        # barrier timeout fails the communicator (later calls answer HCCL_E_SUSPENDING), so the one-sided rows come
        # last, after their RCCL twins have left the digests they are compared with.
        for algo, blocks in ((H.Algo.MESH_CHUNK, 0), (H.Algo.MESH_TWOSHOT, 0), (H.Algo.RING, 0), (H.Algo.RHD, 0),
                             (H.Algo.NHR, 0), (H.Algo.MESH_ONESHOT, 0), (H.Algo.IPC, 0), (H.Algo.IPC, 256),
                             (H.Algo.IPC_TWOSHOT, 0)):
            name = algo.name if blocks == 0 else f"{algo.name}_{blocks}_BLOCKS"
            comm.set_algo(algo)
            comm.set_ipc_blocks(blocks)
            try:
                # two warm-up calls: the eager first call and the graph capture of the second stay out of the timing
                t = _timed(lambda: comm.all_reduce(send, recv, H.HcclReduceOp.SUM, s), 3, warmup=2)
            except H.HcclError as e:  # one schedule failing never hides the others
                out[name] = {"error": str(e)}
                continue
            row = {"ms": round(t * 1e3, 3), "busbw_GBps": round(C3_BYTES / t / 1e9 * 2 * (world - 1) / world, 2),
                   "ran": H.Algo(comm.last_algo).name}  # an IPC row reads MESH_* if the IPC set-up fell back
            row["xgmi_frac"] = _xgmi_frac(row["busbw_GBps"], world)
            digests.setdefault(algo, recv.view(torch.int32)[:: 1 << 12].clone())
            digest = recv.view(torch.int32)[:: 1 << 12].clone()
            if algo in twin and twin[algo] in digests:
                same = torch.tensor([1 if torch.equal(digests[twin[algo]], digest) else 0], dtype=torch.int32)
                dist.all_reduce(same, op=dist.ReduceOp.MIN)
                # a twin that did not run its own schedule (the one-GPU harness runs every RCCL schedule on the
                # one-sided kernel's auto family) computed another order: no comparison
                twin_ran = out.get(twin[algo].name, {}).get("ran")
                row[f"matches_{twin[algo].name.lower()}"] = bool(same.item()) if twin_ran == twin[algo].name else None
                if twin_ran != twin[algo].name:
                    row["twin_ran"] = twin_ran
                st = comm.ipc_status()
                row["barrier_timeouts"] = st & 1
                row["longest_wait_polls_log2"] = (st >> 8) & 0xFF
            out[name] = row
        # the headline's schedule with every call eager (no executor graph: Config.GRAPH_CACHE 0), beside the default,
        # which replays one captured graph per repeated call
        comm.set_algo(H.Algo.RING)
        comm.set_ipc_blocks(0)
        saved = comm.get_config(H.Config.GRAPH_CACHE)
        comm.set_config(H.Config.GRAPH_CACHE, 0)
        try:
            t = _timed(lambda: comm.all_reduce(send, recv, H.HcclReduceOp.SUM, s), 3, warmup=2)
            out["RING_EAGER"] = {"ms": round(t * 1e3, 3),
                                 "busbw_GBps": round(C3_BYTES / t / 1e9 * 2 * (world - 1) / world, 2),
                                 "ran": H.Algo(comm.last_algo).name, "graph_cache": 0}
        except H.HcclError as e:
            out["RING_EAGER"] = {"error": str(e)}
        finally:
            comm.set_config(H.Config.GRAPH_CACHE, saved)
    finally:
        comm.set_algo(H.Algo.AUTO)
        comm.set_ipc_blocks(0)
    return out


class _stdout_to_stderr:
    """Points file descriptor 1 at stderr for the duration (native libraries that print on stdout: gloo's connection
    report), so that stdout carries nothing but the result line."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False


def _transport_info() -> dict:
    """What the N > 1 numbers were taken with: the RCCL build torch carries (the process's librccl) and any NCCL_* /
    RCCL_* / HCCL_* settings in the environment."""
    try:
        v = torch.cuda.nccl.version()
        ver = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception as e:  # noqa: BLE001
        ver = f"unknown ({type(e).__name__})"
    env = {k: v for k, v in sorted(os.environ.items()) if k.startswith(("NCCL_", "RCCL_", "HCCL_"))}
    return {"rccl_version": ver, "env": env, "p2p_channels": _p2p_channels_info()}


_RCCL_INIT_LOG = None  # NCCL_DEBUG_FILE pattern set by _capture_rccl_init (None: not captured)


def _capture_rccl_init(rank: int) -> None:
    """Before the first RCCL communicator: RCCL's INIT-subsystem log to a file of its own (only when the caller set no
    NCCL_DEBUG), so the line can report the p2p channels RCCL actually set up."""
    global _RCCL_INIT_LOG
    if "NCCL_DEBUG" in os.environ or "NCCL_DEBUG_FILE" in os.environ:
        return
    import tempfile
    _RCCL_INIT_LOG = os.path.join(tempfile.gettempdir(), f"hccl_amd_rccl_init_r{rank}.%p.log")
    os.environ["NCCL_DEBUG"] = "INFO"
    os.environ["NCCL_DEBUG_SUBSYS"] = "INIT"  # not COLL: that logs every call and would load the timed loop
    os.environ["NCCL_DEBUG_FILE"] = _RCCL_INIT_LOG


def _p2p_channels_info() -> dict:
    """The per-peer p2p channels the library configured (HcclAmdRcclP2pChannels) and what RCCL's INIT log reported
    for this rank's communicators ("%d p2p channels, %d p2p channels per peer"; RCCL reports twice the per-peer
    setting: 8 for NCCL_NCHANNELS_PER_PEER=4, profiles/r04_rccl_init_log_probe.txt)."""
    import re
    out = {}
    try:
        per, mn = H.rccl_p2p_channels()
        out["configured"] = {"NCCL_NCHANNELS_PER_PEER": per, "NCCL_MIN_P2P_NCHANNELS": mn}
    except Exception as e:  # noqa: BLE001
        out["configured"] = {"error": f"{type(e).__name__}: {e}"}
    if _RCCL_INIT_LOG is not None:
        path = _RCCL_INIT_LOG.replace("%p", str(os.getpid()))
        try:
            txt = open(path).read()
            rep = [{"p2p_channels": int(a), "per_peer": int(b)}
                   for a, b in re.findall(r"(\d+) p2p channels, (\d+) p2p channels per peer", txt)]
            out["rccl_reported"] = rep[:4]
        except OSError as e:
            out["rccl_reported"] = {"error": str(e)}
    return out


def bench_allreduce(args, rank: int, world: int, local_rank: int) -> dict:
    """Runs the N > 1 measurement on a dedicated stream: every HCCL call gets a real stream (the null default stream
    is rejected with HCCL_E_PTR, as the reference's entry check does) and every event is recorded on it."""
    if os.environ.get("HCCL_AMD_BENCH_HOST_EXCHANGE") == "1":
        local_rank = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank)
    with torch.cuda.stream(torch.cuda.Stream()):
        return _bench_allreduce(args, rank, world, local_rank)


def _failed_line(args, world: int, rank: int, code: int, after_s: float, fallback) -> dict:
    """The line of an N > 1 run whose headline loop failed (a rank's communicator timed out or errored). Every rank
    then exits with EXIT_FAILED after rank 0 printed it, so the failure shows in the run's exit code too."""
    import torch.distributed as dist

    global _EXIT_CODE
    _EXIT_CODE = EXIT_FAILED
    try:
        name = H.HcclResult(code).name
    except ValueError:
        name = str(code)
    dist.destroy_process_group()
    if rank != 0:
        return None
    return {"metric": "device-resident reduce GiB/s (fp32 sum) vs HBM peak; ring all-reduce bus GB/s", "value": 0.0,
            "unit": "GiB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": None,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic (uniform [-1,1) fp32, device-generated)",
            "config": {"workload": "C3: HcclAllReduce fp32 SUM, 4 GiB per rank", "bytes_per_rank": C3_BYTES,
                       "parallelism": f"allreduce x{world}"},
            "error": {"code": name, "after_s": round(after_s, 1), "exec_timeout_s": os.environ.get("HCCL_EXEC_TIMEOUT"),
                      "note": "the headline loop failed on some rank (HcclGetCommAsyncError / entry code, max over "
                              "ranks): an execution timeout aborts the communicator instead of hanging"},
            "headline_fallback": fallback, "transport": _transport_info()}


def _bench_allreduce(args, rank: int, world: int, local_rank: int) -> dict:
    import torch.distributed as dist

    # HCCL_AMD_BENCH_HOST_EXCHANGE=1 is a harness mode for a one-GPU box: every rank shares the device and the
    # communicator is the IPC-only one (HcclAmdCommInitHostExchange, bootstrapped over the gloo group), so the N > 1
    # code path runs end to end; the RCCL-dependent rows then report HCCL_E_NOT_SUPPORT. Never used for results.
    harness = os.environ.get("HCCL_AMD_BENCH_HOST_EXCHANGE") == "1"
    # HCCL_AMD_BENCH_SELFLOOP=1 is the RCCL stand-in on a one-GPU box: one process runs rank 0 of
    # a `world`-rank run on a self-loop communicator (HcclAmdCommInitSelfLoop: rank 0's schedules through a one-rank
    # RCCL communicator, every peer mapped onto itself), so every RCCL-path row of the N > 1 line (the ring headline,
    # c3_schedules, fold_piece, c4, c5, the e2e bucket, RCCL's own all_reduce) runs its code path through RCCL's
    # kernels before any 8-GPU node does. The data no longer means the collective: no result check, never a result.
    selfloop = os.environ.get("HCCL_AMD_BENCH_SELFLOOP") == "1"
    dist_world, dist_rank = (1, 0) if selfloop else (world, rank)
    if harness:
        local_rank = local_rank % max(1, torch.cuda.device_count())
        args.no_rccl_ref = True
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    with _stdout_to_stderr():  # gloo announces its connections on stdout, which carries only the JSON line
        # a rank lost on the host ends the others' gloo waits after 10 minutes, not gloo's default 30
        dist.init_process_group("gloo", rank=dist_rank, world_size=dist_world,
                                timeout=datetime.timedelta(seconds=600))

    def _all_gather(b):
        out = [None] * dist_world
        dist.all_gather_object(out, b)
        return out

    def new_comm():
        if harness:
            return H.comm_init_host_exchange(world, rank, _all_gather)
        if selfloop:
            return H.comm_init_selfloop(world, 0)
        # root info out of band, exactly as the reference's callers do (examples/.../01_allreduce/main.cc:122-136)
        obj = [H.get_root_info() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        return H.comm_init_root_info(world, obj[0], rank)

    if not harness:
        _capture_rccl_init(rank)
    # device memory outside torch's allocator before the communicator and after its first calls (the cost
    # of the p2p channel setting, RCCL's per-peer buffers, plus this library's staging and scratch)
    mem0 = _device_memory_outside_torch()
    comm = new_comm()
    count = C3_BYTES // 4
    g = torch.Generator(device=dev).manual_seed(0x5EED0003 + rank)
    send = torch.rand(count, device=dev, generator=g).mul_(2).sub_(1)
    recv = torch.empty_like(send)
    # C3 as BASELINE.json names it: the ring AllReduce (7 arc-disjoint rings over every xGMI link at n = 8). The
    # reference's own selection at this size (MeshChunk, order O6) and every other family run beside it in
    # other_configs.c3_schedules.
    headline = H.Algo[(args.algo or "ring").upper()]
    stream = torch.cuda.current_stream()

    def warm(c, algo):
        # at least two untimed calls: a shape's first call runs eagerly (RCCL connects the program's peers) and its
        # second captures the executor graph that later calls replay (HCCL_AMD_GRAPH_CACHE), so with fewer the capture
        # would land inside the timed steps
        c.set_algo(algo)
        for _ in range(max(args.warmup, 2)):
            c.all_reduce(send, recv, H.HcclReduceOp.SUM, stream)
        torch.cuda.synchronize()

    # A schedule that errors on its first run on this node must not cost the whole line: every rank agrees (over gloo)
    # and the headline falls back to the reference's own selection on a fresh communicator, with the error recorded.
    fallback = None
    err = ""
    try:
        warm(comm, headline)
        mine = 1
    except H.HcclError as e:
        mine, err = 0, str(e)
    flag = torch.tensor([mine], dtype=torch.int32)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if not flag.item():
        fallback = {"headline_failed": headline.name, "error": err or "on another rank", "measured": "AUTO"}
        try:
            comm.destroy()
        except H.HcclError:
            pass
        comm = new_comm()
        headline = H.Algo.AUTO
        warm(comm, headline)
    dist.barrier()
    torch.cuda.synchronize()
    comm_mem = torch.tensor([_device_memory_outside_torch() - mem0, comm.device_bytes()], dtype=torch.float64)
    dist.all_reduce(comm_mem, op=dist.ReduceOp.MAX)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    e0, e1 = evs[0], evs[-1]
    t0 = time.perf_counter()
    e0.record(stream)
    # The timed loop is bounded: a rank whose peer is lost has its communicator aborted by the library's watchdog
    # past HCCL_EXEC_TIMEOUT (main() sets 120 s unless given), the synchronize then returns, and the line reports the
    # error instead of the run hanging until the driver kills it.
    loop_err = 0
    try:
        for k in range(args.steps):
            comm.all_reduce(send, recv, H.HcclReduceOp.SUM, stream)
            evs[k + 1].record(stream)
    except H.HcclError as e:
        loop_err = e.code
    torch.cuda.synchronize()
    loop_err = loop_err or comm.async_error()
    bad = torch.tensor([loop_err], dtype=torch.int32)
    dist.all_reduce(bad, op=dist.ReduceOp.MAX)
    if bad.item():
        return _failed_line(args, world, rank, int(bad.item()), time.perf_counter() - t0, fallback)
    dist.barrier()
    wall = time.perf_counter() - t0
    # per-step durations (median and p10/p90), each step's max over ranks
    steps_ms = torch.tensor([evs[k].elapsed_time(evs[k + 1]) for k in range(args.steps)], dtype=torch.float64)
    dist.all_reduce(steps_ms, op=dist.ReduceOp.MAX)
    t = torch.tensor([e0.elapsed_time(e1) / 1e3, wall], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t[0])
    per_step = elapsed / args.steps
    algbw = C3_BYTES / per_step / 1e9
    busbw = algbw * 2 * (world - 1) / world
    xgmi_peak = min(world - 1, 7) * XGMI_LINK_GBPS
    value = world * C3_BYTES * args.steps / elapsed / GIB
    algo = comm.last_algo
    # correctness of the measured path at the measured size, right after the timed region and before anything else
    # runs on the communicator: integer-valued inputs make every order exact, so the timed schedule must return
    # exactly sum_r((i % 251) + r) on every rank (checked on the GPU, AND over ranks)
    check = torch.arange(count, device=dev, dtype=torch.int64) % 251
    send.copy_(check + rank)
    comm.set_algo(headline)
    comm.all_reduce(send, recv, H.HcclReduceOp.SUM, stream)
    verified_algo = H.Algo(comm.last_algo).name
    torch.cuda.synchronize()
    ok = torch.tensor([1 if torch.equal(recv, (check * world + world * (world - 1) // 2).to(recv.dtype)) else 0])
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    result_ok = None if selfloop else bool(ok.item())  # a self loop's data does not mean the AllReduce
    del check
    graph_launches, graph_captures = comm.graph_stats()
    comm.destroy()
    g = torch.Generator(device=dev).manual_seed(0x5EED0003 + rank)
    send.copy_(torch.rand(count, device=dev, generator=g).mul_(2).sub_(1))
    res = {
        "metric": "device-resident reduce GiB/s (fp32 sum) vs HBM peak; ring all-reduce bus GB/s",
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(per_step * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (uniform [-1,1) fp32, device-generated)" + (
            "; HARNESS MODE (all ranks on one GPU, IPC-only communicator): not a result" if harness else "") + (
            f"; STAND-IN MODE (one GPU: rank 0's {world}-rank programs over a one-rank RCCL self loop): not a result"
            if selfloop else ""),
        "config": {
            "workload": "C3: HcclAllReduce fp32 SUM, 4 GiB per rank, RCCL send/recv over xGMI + HIP reduce kernels",
            "bytes_per_rank": C3_BYTES,
            "parallelism": f"allreduce x{world}",
            "algorithm": H.Algo(algo).name if algo >= 0 else None,
        },
        "busbw_GBps": round(busbw, 2),
        "algbw_GBps": round(algbw, 2),
        "step_ms": {"median": round(float(np.median(steps_ms.numpy())), 3),
                    "p10": round(float(np.percentile(steps_ms.numpy(), 10)), 3),
                    "p90": round(float(np.percentile(steps_ms.numpy(), 90)), 3),
                    "note": "per-step HIP-event durations on the launch stream, max over ranks per step"},
        "transport": dict(_transport_info(), device_memory={
            "library_GiB": round(float(comm_mem[1]) / GIB, 3),
            # ranks sharing one GPU (the harness) see each other's tensors in the device-wide figure: none then
            "device_outside_torch_GiB": None if harness else round(float(comm_mem[0]) / GIB, 3),
            "note": "library_GiB: the bytes this library holds for the headline communicator after its warm-up "
                    "(HcclAmdCommDeviceBytes: executor staging + the one-sided kernel's allocations), max over ranks; "
                    "device_outside_torch_GiB: device memory in use outside torch's caching allocator after the warm-up "
                    "minus before the communicator (adds RCCL's per-peer channel buffers), max over ranks"}),
        "executor_graphs": {"launches": graph_launches, "captures": graph_captures,
                            "note": "rank 0's calls served by one hipGraphLaunch of the captured executor program "
                                    "(HCCL_AMD_GRAPH_CACHE); the first call of a shape runs eagerly"},
        "per_gpu": {"workload": "C3", "bytes_per_gpu_per_step": C3_BYTES, "algbw_GBps": round(algbw, 2),
                    "busbw_GBps": round(busbw, 2), "bound": "xgmi", "roofline_peak_GBps": round(xgmi_peak, 1),
                    "frac": None if (harness or selfloop) else round(busbw / xgmi_peak, 4)},
        "result_ok": result_ok,
        "result_ok_algorithm": verified_algo,
        "headline_fallback": fallback,
        "rccl_allreduce_reference": None,
        "other_configs": {},
        "roofline": {
            "bound": "xgmi",
            "achieved": round(busbw, 2),
            "peak": round(xgmi_peak, 1),
            "unit": "GB/s",
            # one shared GPU has no xGMI in the path
            "frac": None if (harness or selfloop) else round(busbw / xgmi_peak, 4),
            "traffic": None,
            "note": f"busbw = algbw*2(n-1)/n against the {world - 1} direct xGMI links a rank has to its peers "
                    "x 76.8 GB/s per direction (fully connected node: one link per peer)",
        },
    }
    if selfloop:
        res["n_gpus"] = 1
        res["config"]["parallelism"] = f"self loop standing in for rank 0 of {world}"
        res["stand_in"] = {"virtual_ranks": world, "physical_gpus": 1,
                           "note": "HCCL_AMD_BENCH_SELFLOOP=1: every RCCL-path row of the N > 1 line runs its code "
                                   "through RCCL's kernels on one GPU; times and data are the self loop's, not xGMI's"}
    # Secondary configs and the RCCL reference run under a watchdog: a collective that never returns there (a first
    # run of some schedule on real hardware) must not cost the headline line. At the deadline every rank stops, rank
    # 0 printing the result with what finished so far.
    extra = res["other_configs"]
    wd = _Watchdog(float(os.environ.get("HCCL_AMD_BENCH_EXTRAS_DEADLINE_S", "300")), rank, res)
    wd.start()
    if not args.no_extra_configs:
        # Each secondary config gets a communicator of its own: a failure in one (say an IPC barrier timeout, after
        # which the communicator answers HCCL_E_SUSPENDING) cannot take the others, or the headline, with it.
        for name, fn in (("c3_schedules", lambda cm: bench_c3_algos(cm, send, recv, world)),
                         ("fold_piece", lambda cm: bench_fold_piece(cm, send, recv, world)),
                         ("c4", lambda cm: bench_c4(cm, send, recv, world)),
                         ("c5", lambda cm: bench_c5(cm, send, recv, world)),
                         ("end_to_end_host_buffers", lambda cm: bench_e2e_allreduce(cm, world))):
            wd.stage(name)
            cm = None
            try:
                cm = new_comm()
                extra[name] = fn(cm)
            except Exception as e:  # noqa: BLE001  (a secondary config never hides the headline line)
                extra[name] = {"error": f"{type(e).__name__}: {e}"}
            finally:
                if cm is not None:
                    try:
                        cm.destroy()
                    except Exception as e:  # noqa: BLE001
                        extra.setdefault(name, {})["destroy_error"] = f"{type(e).__name__}: {e}"
    try:
        extra["data_path_choice"] = recommend_data_paths(extra.get("c3_schedules"), extra.get("c5"))
    except Exception as e:  # noqa: BLE001
        extra["data_path_choice"] = {"error": f"{type(e).__name__}: {e}"}
    if not args.no_rccl_ref:
        wd.stage("rccl_allreduce_reference")
        res["rccl_allreduce_reference"] = rccl_allreduce_reference(send, recv, dist_world, args)
    if not args.no_cpu_baseline and rank == 0:
        # the reference's CPU path on this box's host cores, beside the line (BASELINE.json north_star): the C2 leg
        # and this N's AllReduce program replayed on the host at a stated size
        wd.stage("cpu_baseline")
        try:
            cb = cpu_baseline_allreduce(world, int(headline))
            cb["c2"] = cpu_baseline_c2(args.cpu_budget)
            res["cpu_baseline"] = cb
        except Exception as e:  # noqa: BLE001
            res["cpu_baseline"] = {"error": f"{type(e).__name__}: {e}"}
    wd.cancel()
    dist.destroy_process_group()
    return res if rank == 0 else None


_PRINTED = threading.Event()
_PRINT_LOCK = threading.Lock()
# Exit codes besides 0: the headline loop failed on some rank (the line carries "error"), the extras watchdog
# stopped the run (the line carries "watchdog"), or the timed path's output was wrong (`result_ok` false). The JSON
# line is printed first in every case.
EXIT_FAILED = 3
EXIT_WATCHDOG = 4
EXIT_WRONG_RESULT = 5
EXIT_REFUSED = 6  # the run's shape does not match the machine or the launch (_refuse); nothing was measured
_EXIT_CODE = 0
METRIC = "device-resident reduce GiB/s (fp32 sum) vs HBM peak; ring all-reduce bus GB/s"


def emit(res: dict) -> None:
    """Prints the one JSON line, once per process (the watchdog and the normal exit may race)."""
    with _PRINT_LOCK:
        if _PRINTED.is_set():
            return
        print(json.dumps(res), flush=True)
        _PRINTED.set()


class _Watchdog:
    """Ends a rank whose secondary configs overrun `seconds`: rank 0 first prints the result (headline plus what
    finished) with a note naming the stage that overran, then every rank exits with EXIT_WATCHDOG. Every rank arms it
    at the same point, so they stop together."""

    def __init__(self, seconds: float, rank: int, res: dict):
        self.seconds, self.rank, self.res, self.current = seconds, rank, res, "start"
        self.t0 = time.perf_counter()
        self.timer = threading.Timer(seconds, self._fire)
        self.timer.daemon = True

    def start(self):
        self.timer.start()

    def stage(self, name: str):
        self.current = name

    def cancel(self):
        self.timer.cancel()

    def _fire(self):
        if self.rank == 0:
            self.res["watchdog"] = {"stopped_at": self.current, "after_s": round(time.perf_counter() - self.t0, 1),
                                    "deadline_s": self.seconds}
            emit(self.res)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(EXIT_WATCHDOG)


def _refuse(args, why: str, world=None) -> None:
    """Prints the refusal line (value null: nothing was measured) and exits with EXIT_REFUSED."""
    print(json.dumps({"metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": args.gpus, "steps": args.steps,
                      "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True, "scaling": "weak",
                      "vs_baseline": None, "dtype": "fp32", "data": "none (refused before any measurement)",
                      "config": {"workload": "C3" if args.gpus > 1 else "C2"},
                      "error": {"refused": why, "world_size_env": world,
                                "device_count": _device_count()}}), flush=True)
    sys.exit(EXIT_REFUSED)


def _device_count() -> int:
    # counting devices does not initialise the GPU on this stack (torch reads the count without creating a context),
    # so the launcher may call it before it starts the ranks
    try:
        return int(torch.cuda.device_count())
    except Exception:  # noqa: BLE001
        return 0


def _harness() -> bool:
    return os.environ.get("HCCL_AMD_BENCH_HOST_EXCHANGE") == "1"


def _free_port() -> int:
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_command(gpus: int, argv, port: int):
    """The command the launcher starts for `bench.py --gpus N` without WORLD_SIZE: one rank per GPU under
    torch.distributed.run on this node, rendezvous on 127.0.0.1, the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]


def launch_ranks(args, argv) -> int:
    """`bench.py --gpus N` (N > 1) started without a launcher: the parent makes no GPU call, starts N rank processes
    (torch.distributed.run) as a child, relays rank 0's JSON line to stdout and everything else to stderr, and exits
    with the child's code. The reference's callers run one rank per device the same way (examples/02_collectives/
    01_allreduce/main.cc:113-136)."""
    import subprocess

    cmd = launch_command(args.gpus, argv, _free_port())
    log("[bench] launching", " ".join(cmd))
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True)
    for line in proc.stdout:
        (sys.stdout if line.startswith("{") else sys.stderr).write(line)
        sys.stdout.flush()
    return proc.wait()


def check_launch(args):
    """The run's shape against the launch and the machine. Returns "launch" when this process
    must start the ranks, "local" for the N = 1 line, "rank" for one rank of an N > 1 run; refuses (exit EXIT_REFUSED,
    one JSON line from rank 0) when --gpus disagrees with WORLD_SIZE, or when the node has fewer GPUs than ranks
    (unless HCCL_AMD_BENCH_HOST_EXCHANGE=1 puts every rank on one GPU, the harness that is never a result)."""
    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus < 1:
        _refuse(args, f"--gpus {args.gpus}: at least one GPU")
    if env_world is None:
        if args.gpus == 1:
            return "local"
        if os.environ.get("HCCL_AMD_BENCH_SELFLOOP") == "1":
            # the RCCL stand-in: this one process runs rank 0 of the --gpus N line over a self loop (never a result)
            if _device_count() < 1:
                _refuse(args, "the self-loop stand-in needs one GPU; this node has none")
            return "selfloop"
        if not _harness() and _device_count() < args.gpus:
            _refuse(args, f"--gpus {args.gpus} but this node has {_device_count()} GPU(s)")
        return "launch"
    world = int(env_world)
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        if rank == 0:
            _refuse(args, f"WORLD_SIZE={world} but --gpus {args.gpus}: one rank per GPU", world)
        sys.exit(EXIT_REFUSED)
    need = 1 if _harness() else world
    if _device_count() < need:
        if rank == 0:
            _refuse(args, f"{world} rank(s) but this node has {_device_count()} GPU(s)", world)
        sys.exit(EXIT_REFUSED)
    return "local" if world == 1 else "rank"


def main():
    import faulthandler

    faulthandler.dump_traceback_later(900, exit=False)  # diagnostics only: stacks to stderr if a run stalls
    # a lost peer ends an IPC launch after this long (status bit 0, sticky per communicator) instead of 60 s, so a
    # failing secondary row cannot stretch the driver's run
    os.environ.setdefault("HCCL_AMD_IPC_TIMEOUT_MS", "10000")
    # the RCCL path's execution bound (the library's watchdog aborts a communicator whose collective has not finished
    # this long after it started): a lost rank ends the N > 1 run with a line
    os.environ.setdefault("HCCL_EXEC_TIMEOUT", "120")
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-e2e", action="store_true", help="skip the host-buffer (PCIe-inclusive) measurement")
    p.add_argument("--no-rccl-ref", action="store_true", help="N>1: skip timing RCCL's own all_reduce beside ours")
    p.add_argument("--no-extra-configs", action="store_true", help="N>1: skip the C4 (RS+AG) and C5 (RHD sweep) lines")
    p.add_argument("--cpu-budget", type=float, default=12.0)
    p.add_argument("--algo", default="", help="N>1: the headline AllReduce schedule (default ring; mesh_chunk is the "
                                              "reference's own selection at 4 GiB, auto, rhd, ipc ...)")
    argv = sys.argv[1:]
    args = p.parse_args(argv)
    mode = check_launch(args)
    if mode == "launch":
        sys.exit(launch_ranks(args, argv))
    if mode == "selfloop":
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        res = bench_allreduce(args, 0, args.gpus, 0)
    elif mode == "rank":
        world = int(os.environ["WORLD_SIZE"])
        rank = int(os.environ["RANK"])
        res = bench_allreduce(args, rank, world, int(os.environ.get("LOCAL_RANK", rank)))
    else:
        res = bench_local(args)
    global _EXIT_CODE
    if res is not None:
        emit(res)
        if res.get("result_ok") is False and _EXIT_CODE == 0:
            _EXIT_CODE = EXIT_WRONG_RESULT
    sys.stdout.flush()
    sys.exit(_EXIT_CODE)


if __name__ == "__main__":
    main()
