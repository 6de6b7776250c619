"""Parity at BASELINE.json's full sizes (configs C3, C4, C5) on a loopback world of 8 ranks on the one GPU, through
properties that do not need the CPU oracle to run at that size:
  * C3, 4 GiB fp32 per rank, two-shot order O2 (ins_temp_all_reduce_mesh_1D_two_shot.cc:327-335) on random data:
    bit-exact against the same left fold done by torch on the GPU (IEEE fp32 adds in the same order), on the RCCL-path
    schedule and on the one-sided IPC kernel;
  * C3 with the reference's own selection (MeshChunk at this size) on integer-valued fp32: exact sums, so every
    element holds every rank exactly once;
  * C4, 2 GiB bf16 per rank: ReduceScatter then AllGather of integer-valued bf16 equals the exact AllReduce;
  * C5's largest point, 4 GiB fp16 per rank on the RHD schedule: integer-valued fp16, exact sums;
  * (r04) C4's MeshChunk ReduceScatter (RCCL path and one-sided kernel) and C5's RHD on random data: bit-exact against
    the same bf16 / fp16 steps (fp32 add, RNE) in the same order done by torch on the GPU;
  * (r04) C3's MeshChunk AllReduce (the reference's selection at 4 GiB) on random fp32: bit-exact against the same
    adds in the same order (executor loops, n-1 sub-slices per chunk, owner then O6 peers).
Each random-data test first asserts that the plain rank-order fold differs from the closed form on its data, so a pass
pins the association order and not only the sum.
The small-size tests pin the association order of every family bit for bit against the oracle; these pin that
nothing changes at the sizes the benchmark runs.
"""
import threading

import pytest
import torch

import hccl_amd as H

pytestmark = pytest.mark.gpu

N = 8


@pytest.fixture(scope="module")
def world():
    comms = H.loopback_world(N)
    yield comms
    torch.cuda.synchronize()
    for c in comms:
        c.destroy()


def run_all(comms, fn):
    errs = []
    streams = [torch.cuda.Stream() for _ in comms]

    def body(r):
        try:
            fn(r, streams[r])
        except Exception as e:  # noqa: BLE001
            errs.append((r, e))

    torch.cuda.synchronize()
    th = [threading.Thread(target=body, args=(r,)) for r in range(len(comms))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=900)
    torch.cuda.synchronize()
    assert not errs, errs


def pattern(count, r, dtype, mod):
    """Small integers, exact in `dtype` and in every partial sum over 8 ranks: (i % mod) + r."""
    return (torch.arange(count, device="cuda", dtype=torch.int64) % mod + r).to(dtype)


@pytest.mark.parametrize("algo", [H.Algo.MESH_TWOSHOT, H.Algo.IPC_TWOSHOT])
def test_c3_full_size_two_shot_bit_exact_random(world, algo):
    count = (4 << 30) // 4
    xs = []
    for r in range(N):
        g = torch.Generator(device="cuda").manual_seed(0xC3 + r)
        xs.append(torch.rand(count, device="cuda", generator=g).mul_(2).sub_(1))
    want = xs[0].clone()
    for r in range(1, N):
        want.add_(xs[r])  # acc = x_r + acc, r ascending (order O2)
    outs = [torch.empty(count, device="cuda") for _ in range(N)]
    for c in world:
        c.set_algo(algo)
    try:
        run_all(world, lambda r, s: world[r].all_reduce(xs[r], outs[r], H.HcclReduceOp.SUM, s))
        assert world[0].last_algo == algo
        for r in range(N):
            bad = torch.count_nonzero(outs[r].view(torch.int32) != want.view(torch.int32)).item()
            assert bad == 0, (r, bad)
    finally:
        for c in world:
            c.set_algo(H.Algo.AUTO)
    del xs, outs, want


def _bounds(count, parts, es=4):
    """tests/sched_ref.py chunk_bounds: ceil split rounded up to 128 B."""
    align = 128 // es
    sc = -(-count // parts)
    sc = -(-sc // align) * align
    return [(min(count, c * sc), min(count, c * sc + sc)) for c in range(parts)]


def test_c3_full_size_ring_bit_exact_random(world):
    """C3 as BASELINE.json names it: the ring AllReduce, 8 ranks x 4 GiB fp32, random data. The schedule runs the 7
    arc-disjoint rings of HcclAmdRingTable(8) at once, part k of the buffer on ring k; the chunk at ring position c
    ends as acc = x_{cyc[c+1]}, then acc = acc + x_{cyc[c+j]} for j = 2 .. n (tests/sched_ref.py allreduce_ring).
    The same IEEE fp32 adds in the same order are done by torch on the GPU: the outputs must be identical bits."""
    count = (4 << 30) // 4
    xs = []
    for r in range(N):
        g = torch.Generator(device="cuda").manual_seed(0xC3A + r)
        xs.append(torch.rand(count, device="cuda", generator=g).mul_(2).sub_(1))
    rings = H.ring_table(N)
    assert len(rings) == N - 1
    want = torch.empty(count, device="cuda")
    for k, (pb, pe) in enumerate(_bounds(count, len(rings))):
        cyc = rings[k]
        for c, (b, e) in enumerate(_bounds(pe - pb, N)):
            if e <= b:
                continue
            sl = slice(pb + b, pb + e)
            acc = xs[cyc[(c + 1) % N]][sl].clone()
            for j in range(2, N + 1):
                acc.add_(xs[cyc[(c + j) % N]][sl])
            want[sl] = acc
    outs = [torch.empty(count, device="cuda") for _ in range(N)]
    for c in world:
        c.set_algo(H.Algo.RING)
    try:
        run_all(world, lambda r, s: world[r].all_reduce(xs[r], outs[r], H.HcclReduceOp.SUM, s))
        assert world[0].last_algo == H.Algo.RING
        for r in range(N):
            bad = torch.count_nonzero(outs[r].view(torch.int32) != want.view(torch.int32)).item()
            assert bad == 0, (r, bad)
    finally:
        for c in world:
            c.set_algo(H.Algo.AUTO)
    del xs, outs, want


def test_c3_full_size_reference_selection_exact(world):
    count = (4 << 30) // 4
    xs = [pattern(count, r, torch.float32, 251) for r in range(N)]
    outs = [torch.empty(count, device="cuda") for _ in range(N)]
    run_all(world, lambda r, s: world[r].all_reduce(xs[r], outs[r], H.HcclReduceOp.SUM, s))
    assert world[0].last_algo == H.Algo.MESH_CHUNK  # bytes * 8 / n^2 > 32 MiB (all_reduce_auto_selector.cc)
    want = pattern(count, 0, torch.float32, 251).mul_(N).add_(N * (N - 1) // 2)
    for r in range(N):
        assert torch.equal(outs[r], want), r
    del xs, outs, want


def test_c4_full_size_reduce_scatter_then_all_gather(world):
    count = (2 << 30) // 2
    shard = count // N
    xs = [pattern(count, r, torch.bfloat16, 29) for r in range(N)]
    shards = [torch.empty(shard, dtype=torch.bfloat16, device="cuda") for _ in range(N)]
    fulls = [torch.empty(count, dtype=torch.bfloat16, device="cuda") for _ in range(N)]
    run_all(world, lambda r, s: world[r].reduce_scatter(xs[r], shards[r], H.HcclReduceOp.SUM, s))
    rs_algo = world[0].last_algo
    run_all(world, lambda r, s: world[r].all_gather(shards[r], fulls[r], s))
    want = pattern(count, 0, torch.float32, 29).mul_(N).add_(N * (N - 1) // 2).to(torch.bfloat16)
    for r in range(N):
        assert torch.equal(shards[r], want[r * shard:(r + 1) * shard]), (r, rs_algo)
        assert torch.equal(fulls[r], want), r
    del xs, shards, fulls, want


def test_c5_largest_point_rhd_exact(world):
    count = (4 << 30) // 2
    xs = [pattern(count, r, torch.float16, 61) for r in range(N)]
    outs = [torch.empty(count, dtype=torch.float16, device="cuda") for _ in range(N)]
    for c in world:
        c.set_algo(H.Algo.RHD)
    try:
        run_all(world, lambda r, s: world[r].all_reduce(xs[r], outs[r], H.HcclReduceOp.SUM, s))
        assert world[0].last_algo == H.Algo.RHD
        want = pattern(count, 0, torch.float32, 61).mul_(N).add_(N * (N - 1) // 2).to(torch.float16)
        for r in range(N):
            assert torch.equal(outs[r], want), r
    finally:
        for c in world:
            c.set_algo(H.Algo.AUTO)
    del xs, outs


def _o6_peers(n, t, j):
    """tests/sched_ref.py o6_peers: senders into sub-slice j of owner t, step by step."""
    out = []
    for s in range(n - 1):
        x = s + j + 1
        if x >= n:
            x += 1
        out.append((t + x) % n)
    return out


def _rs_subslices(count, parts, es):
    """tests/sched_ref.py rs_subslices (…meshchunk.cc:155-180): 4-KiB aligned sub-slices, the rest last."""
    align = count * es // parts // 4096 * 4096
    if parts < 2 or align == 0:
        base, big = divmod(count, parts)
        out, b = [], 0
        for i in range(parts):
            ln = base + (1 if i < big else 0)
            out.append((b, b + ln))
            b += ln
        return out
    a = align // es
    return [(i * a, (i + 1) * a) for i in range(parts - 1)] + [((parts - 1) * a, count)]


@pytest.mark.parametrize("algo", [H.Algo.AUTO, H.Algo.IPC])
def test_c4_full_size_reduce_scatter_meshchunk_bf16_random(world, algo):
    """C4 as named: ReduceScatter of 2 GiB bf16 per rank on 8 ranks, random data, the reference's own selection
    (MeshChunk: order O6 per 4-KiB sub-slice, per executor loop of min(ccl - 1 MiB, (ccl - 1 MiB) / (n-1)) bytes,
    ins_temp_reduce_scatter_mesh_1D_meshchunk.cc, ins_v2_reduce_scatter_sole_executor.cc:160-175) on the RCCL-path
    schedule and on the one-sided kernel (HCCL_AMD_ALGO_IPC, same family): bit-exact against the same bf16 adds
    (fp32 add, round to nearest even) in the same order done by torch on the GPU (tests/sched_ref.py
    reduce_scatter_meshchunk restated for torch); then AllGather of the shards is every shard in rank order."""
    count = (2 << 30) // 2
    rc = count // N
    es = 2
    xs = []
    for r in range(N):
        g = torch.Generator(device="cuda").manual_seed(0xC4 + r)
        xs.append(torch.rand(count, device="cuda", generator=g).mul_(2).sub_(1).to(torch.bfloat16))
    ccl = 200 << 20
    tmp = ccl - (1 << 20)
    per = max(1, min(tmp, tmp // (N - 1) // 128 * 128) // es)
    want = [torch.empty(rc, dtype=torch.bfloat16, device="cuda") for _ in range(N)]
    for off in range(0, rc, per):
        cnt = min(per, rc - off)
        for t in range(N):
            for j, (sb, se) in enumerate(_rs_subslices(cnt, N - 1, es)):
                if se <= sb:
                    continue
                lo, hi = t * rc + off + sb, t * rc + off + se
                acc = xs[t][lo:hi].clone()
                for q in _o6_peers(N, t, j):
                    acc = xs[q][lo:hi] + acc  # bf16: fp32 add, RNE
                want[t][off + sb:off + se] = acc
    o2 = xs[0][:rc].clone()  # the order matters on this data (rank 0's shard, plain rank-order fold)
    for r in range(1, N):
        o2 = xs[r][:rc] + o2
    assert torch.count_nonzero(o2.view(torch.int16) != want[0].view(torch.int16)).item() > 0
    del o2
    shards = [torch.empty(rc, dtype=torch.bfloat16, device="cuda") for _ in range(N)]
    for c in world:
        c.set_algo(algo)
    try:
        run_all(world, lambda r, s: world[r].reduce_scatter(xs[r], shards[r], H.HcclReduceOp.SUM, s))
        used = world[0].last_algo
        assert used == (H.Algo.MESH_CHUNK if algo == H.Algo.AUTO else H.Algo.IPC), used
        for r in range(N):
            bad = torch.count_nonzero(shards[r].view(torch.int16) != want[r].view(torch.int16)).item()
            assert bad == 0, (r, bad)
        del xs
        fulls = [torch.empty(count, dtype=torch.bfloat16, device="cuda") for _ in range(N)]
        run_all(world, lambda r, s: world[r].all_gather(shards[r], fulls[r], s))
        cat = torch.cat(shards)
        for r in range(N):
            assert torch.equal(fulls[r].view(torch.int16), cat.view(torch.int16)), r
    finally:
        for c in world:
            c.set_algo(H.Algo.AUTO)


def test_c5_largest_point_rhd_fp16_random(world):
    """C5's largest point as named: RHD AllReduce of 4 GiB fp16 per rank on 8 ranks, random data: bit-exact against
    the RHD closed form done by torch on the GPU. The buffer is split into the schedule's concurrent instances (128-B
    aligned ceil parts, instance j on virtual ranks table[j]); an element of chunk v of part j is the recursive-halving
    tree over the operands of virtual ranks v ^ q: at distance M = 4, 2, 1 leaf q takes leaf q + M (op) leaf q (fp16:
    fp32 add, round to nearest even; tests/sched_ref.py allreduce_rhd / rhd_virtual)."""
    count = (4 << 30) // 2
    es = 2
    xs = []
    for r in range(N):
        g = torch.Generator(device="cuda").manual_seed(0xC5 + r)
        xs.append(torch.rand(count, device="cuda", generator=g).mul_(2).sub_(1).to(torch.float16))
    table = H.rhd_table(N)
    nbytes = count * es
    inst = 1
    while inst < N - 1 and (inst + 1) ** 2 * (1 << 20) <= 2 * nbytes:
        inst += 1
    table = table[:inst]
    want = torch.empty(count, dtype=torch.float16, device="cuda")
    for j, (pb, pe) in enumerate(_bounds(count, len(table), es)):
        for v, (b, e) in enumerate(_bounds(pe - pb, N, es)):
            if e <= b:
                continue
            sl = slice(pb + b, pb + e)
            leaves = [xs[table[j][v ^ q]][sl] for q in range(N)]
            m = N // 2
            while m >= 1:
                leaves = [leaves[q + m] + leaves[q] for q in range(m)]
                m //= 2
            want[sl] = leaves[0]
    o2 = xs[0].clone()  # the order matters on this data: the plain rank-order fold differs somewhere
    for r in range(1, N):
        o2 = xs[r] + o2
    assert torch.count_nonzero(o2.view(torch.int16) != want.view(torch.int16)).item() > 0
    del o2
    outs = [torch.empty(count, dtype=torch.float16, device="cuda") for _ in range(N)]
    for c in world:
        c.set_algo(H.Algo.RHD)
    try:
        run_all(world, lambda r, s: world[r].all_reduce(xs[r], outs[r], H.HcclReduceOp.SUM, s))
        assert world[0].last_algo == H.Algo.RHD
        for r in range(N):
            bad = torch.count_nonzero(outs[r].view(torch.int16) != want.view(torch.int16)).item()
            assert bad == 0, (r, bad)
    finally:
        for c in world:
            c.set_algo(H.Algo.AUTO)
    del xs, outs, want


@pytest.mark.parametrize("algo", [H.Algo.AUTO, H.Algo.IPC])
def test_c3_full_size_meshchunk_random(world, algo):
    """C3 with the reference's own selection at 4 GiB fp32 per rank (MeshChunk AllReduce, order O6), random data, on
    the RCCL-path schedule and on the one-sided kernel: bit-exact against torch's fp32 adds in the closed form of
    tests/sched_ref.py allreduce_meshchunk (executor loops of min(ccl, ccl / 2) rounded down to 128 B, chunks of
    ceil(cnt / n) elements, n - 1 even sub-slices per chunk, owner first then o6_peers per sub-slice)."""
    count = (4 << 30) // 4
    es = 4
    xs = []
    for r in range(N):
        g = torch.Generator(device="cuda").manual_seed(0xC36 + r)
        xs.append(torch.rand(count, device="cuda", generator=g).mul_(2).sub_(1))
    ccl = 200 << 20
    per = max(1, min(ccl, ccl // 2 // 128 * 128) // es)
    want = torch.empty(count, device="cuda")
    for off in range(0, count, per):
        cnt = min(per, count - off)
        cs = -(-cnt // N)
        for t in range(N):
            b, e = min(cnt, t * cs), min(cnt, (t + 1) * cs)
            base, big = divmod(e - b, N - 1)
            sb = 0
            for j in range(N - 1):
                se = sb + base + (1 if j < big else 0)
                if se > sb:
                    sl = slice(off + b + sb, off + b + se)
                    acc = xs[t][sl].clone()
                    for q in _o6_peers(N, t, j):
                        acc = xs[q][sl] + acc
                    want[sl] = acc
                sb = se
    # the order matters on this data: the plain rank-order fold (O2) differs from the closed form somewhere
    o2 = xs[0].clone()
    for r in range(1, N):
        o2.add_(xs[r])
    assert torch.count_nonzero(o2.view(torch.int32) != want.view(torch.int32)).item() > 0
    del o2
    outs = [torch.empty(count, device="cuda") for _ in range(N)]
    for c in world:
        c.set_algo(algo)
    try:
        run_all(world, lambda r, s: world[r].all_reduce(xs[r], outs[r], H.HcclReduceOp.SUM, s))
        assert world[0].last_algo == (H.Algo.MESH_CHUNK if algo == H.Algo.AUTO else H.Algo.IPC)
        for r in range(N):
            bad = torch.count_nonzero(outs[r].view(torch.int32) != want.view(torch.int32)).item()
            assert bad == 0, (r, bad)
    finally:
        for c in world:
            c.set_algo(H.Algo.AUTO)
    del xs, outs, want
