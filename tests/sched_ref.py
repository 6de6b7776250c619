"""Closed-form expected results of every schedule, written independently of the C++ generators.

Each function returns, for every rank, the output buffer the collective must produce, built from the
association orders of SURVEY.md Appendix A with the oracle's element rule (acc = src (op) dst, where the incoming
or later operand is src, as in the reference's LocalReduce / write-reduce / read-reduce conventions):

  O1  one-shot AllReduce, mesh ReduceScatter, Reduce:  acc = x_me; acc = x_q (op) acc, q ascending, q != me
  O2  two-shot AllReduce:                              acc = x_0;  acc = x_q (op) acc, q = 1 .. n-1
  rings (R arc-disjoint Hamiltonian cycles, part k on ring k; chunk at position c):
      acc = x_{cyc[c+1]}; acc = acc (op) x_{cyc[c+k]}   (the travelling partial is src)
  RHD  pairwise: at distance d the kept half becomes partner_partial (op) my_partial; n-1 instances on virtual ranks
  O6  MeshChunk AllReduce / ReduceScatter, sub-slice j of owner t: acc = x_t; acc = x_{t+o} (op) acc for the rank
      offsets o = j+1 .. n-1, 1 .. j (ins_temp_all_reduce_mesh_1D_two_shot_mesh_chunk.cc:204-275,
      ins_temp_reduce_scatter_mesh_1D_meshchunk.cc:190-252: in step s, sub-slice j of receiver t is written by sender
      t + nextNum, nextNum = s + j + 1, plus one once it reaches n)
"""
import numpy as np

from oracle import oracle as O

ALIGN = 128


UB_MAX_DATA_SIZE = 256 << 20  # alg_param.h:37


def ccl_bytes_from_env():
    """HCCL_BUFFSIZE in MB (default 200), as the library reads it."""
    import os
    v = os.environ.get("HCCL_BUFFSIZE", "")
    try:
        mb = int(v) if v else 200
    except ValueError:
        mb = 200
    return (mb if mb > 0 else 200) << 20


def ref_loops(count, es, transport_bound, scratch_multiple, ccl):
    """Executor loops (ins_v2_all_reduce_sole_executor.cc:160-208, reduce_sole_executor.cc:120-170): at most
    min(transport bound, ccl / multiple rounded down to 128 B) bytes each; the template slices every loop alone."""
    nbytes = transport_bound
    if scratch_multiple:
        nbytes = min(nbytes, ccl // scratch_multiple // ALIGN * ALIGN)
    per = max(1, nbytes // es)
    return [(off, min(per, count - off)) for off in range(0, count, per)]


def balanced_bounds(count, n):
    """ReduceMesh1DTwoShot::CalcSlice (reduce_mesh_1D_two_shot.cc:108-131)."""
    base, rem = divmod(count, n)
    out, b = [], 0
    for c in range(n):
        ln = base + (1 if c < rem else 0)
        out.append((b, b + ln))
        b += ln
    return out


def ceil_bounds(count, n):
    """ReduceNHR::CalcSlice (reduce_nhr.cc:114-138): ceil(count / n) elements, trailing slices short or empty."""
    cs = -(-count // n)
    return [(min(count, c * cs), min(count, (c + 1) * cs)) for c in range(n)]


def floor_bounds(count, n):
    """InsTempAllReduceNHR (ins_temp_all_reduce_nhr.cc:171-173): floor(count / n), the tail on the last slice."""
    se = count // n
    return [(i * se, (i + 1) * se if i < n - 1 else count) for i in range(n)]


def chunk_bounds(count, n, es):
    align = max(1, ALIGN // es)
    sc = -(-count // n)
    sc = -(-sc // align) * align
    out = []
    for c in range(n):
        b = min(count, c * sc)
        e = min(count, b + sc)
        out.append((b, e))
    return out


def fold(dtype, op, arrays):
    return O.reduce_n(dtype, op, [np.ascontiguousarray(a) for a in arrays])


def apply(dtype, op, src, dst):
    """dst' = src (op) dst, returns a new array."""
    return O.local_reduce(dtype, op, np.ascontiguousarray(dst).copy(), np.ascontiguousarray(src))


def allreduce_o1(dtype, op, xs):
    n = len(xs)
    return [fold(dtype, op, [xs[me]] + [xs[q] for q in range(n) if q != me]) for me in range(n)]


def allreduce_o2(dtype, op, xs):
    r = fold(dtype, op, xs)
    return [r.copy() for _ in xs]


def ring_table(n):
    """The library's rings (HcclAmdRingTable); tests/test_schedules.py checks they are arc-disjoint Hamiltonian
    cycles."""
    import hccl_amd as H
    return H.ring_table(n)


def ring_count(n, nbytes):
    """Rings a call uses: the largest R (at most the table's) with R^2 x 2n x 1 MiB <= 13.65 x nbytes, at least 1;
    nbytes = the AllReduce buffer, the ReduceScatter input or the AllGather output of one rank."""
    most = len(ring_table(n))
    r = 1
    while r < most and (r + 1) ** 2 * 2.0 * n * (1 << 20) <= 13.65 * nbytes:
        r += 1
    return r


def ring_parts(count, n_rings, es):
    """Part k of the buffer travels around ring k (ceil split, 128-B aligned, as chunk_bounds)."""
    return chunk_bounds(count, n_rings, es)


def ring_chunk(dtype, op, xs, cyc, c, sl):
    """Chunk at ring position c: acc = x_{cyc[c+1]}; acc = acc (op) x_{cyc[c+k]} (the travelling partial is src)."""
    n = len(xs)
    acc = xs[cyc[(c + 1) % n]][sl].copy()
    for k in range(2, n + 1):
        acc = apply(dtype, op, acc, xs[cyc[(c + k) % n]][sl])
    return acc


def allreduce_ring(dtype, op, xs):
    n = len(xs)
    es = xs[0].itemsize
    rings = ring_table(n)[:ring_count(n, xs[0].size * es)]
    out = np.empty_like(xs[0])
    for k, (pb, pe) in enumerate(ring_parts(xs[0].size, len(rings), es)):
        for c, (b, e) in enumerate(chunk_bounds(pe - pb, n, es)):
            if e > b:
                out[pb + b:pb + e] = ring_chunk(dtype, op, xs, rings[k], c, slice(pb + b, pb + e))
    return [out.copy() for _ in xs]


def rhd_virtual(dtype, op, xs, bounds):
    """Classic RHD on ranks 0..n-1 (partner r ^ d, d = n/2 .. 1; the kept half becomes partner_partial (op) mine),
    then every chunk from its owner. xs are the operands in virtual-rank order; returns the reduced buffer."""
    n = len(xs)
    part = [x.copy() for x in xs]  # each rank's running partial (only its kept region is meaningful)
    lo = [0] * n
    hi = [n] * n
    d = n // 2
    while d >= 1:
        new = [p.copy() for p in part]
        for r in range(n):
            partner = r ^ d
            mid = lo[r] + d
            keep = (lo[r], mid) if (r & d) == 0 else (mid, hi[r])
            b, e = bounds[keep[0]][0], bounds[keep[1] - 1][1]
            if e > b:
                new[r][b:e] = apply(dtype, op, part[partner][b:e], part[r][b:e])
        for r in range(n):
            if (r & d) == 0:
                hi[r] = lo[r] + d
            else:
                lo[r] = lo[r] + d
        part = new
        d //= 2
    out = np.empty_like(xs[0])
    for c, (b, e) in enumerate(bounds):
        if e > b:
            out[b:e] = part[c][b:e]
    return out


def rhd_instances(n, nbytes):
    """Concurrent RHD instances for nbytes per rank: the largest R <= n-1 with R^2 MiB <= 2 x nbytes (at least 1)."""
    r = 1
    while r < max(1, n - 1) and (r + 1) ** 2 * (1 << 20) <= 2 * nbytes:
        r += 1
    return r


def allreduce_rhd(dtype, op, xs):
    """rhd_instances concurrent RHD instances (the first rows of HcclAmdRhdTable): part j runs the classic RHD on
    virtual ranks, virtual rank v being real rank table[j][v]."""
    import hccl_amd as H
    n = len(xs)
    es = xs[0].itemsize
    table = H.rhd_table(n)[:rhd_instances(n, xs[0].size * es)]
    out = np.empty_like(xs[0])
    for j, (pb, pe) in enumerate(chunk_bounds(xs[0].size, len(table), es)):
        if pe > pb:
            virt = [xs[table[j][v]][pb:pe] for v in range(n)]
            out[pb:pe] = rhd_virtual(dtype, op, virt, chunk_bounds(pe - pb, n, es))
    return [out.copy() for _ in xs]


def nhr_steps(n, me, gather):
    """Step lists of ins_temp_all_reduce_nhr.cc:390-482 (GetReduceScatterStepInfoList / GetAllGatherStepInfoList),
    restated from the reference text."""
    n_steps = 0
    t = n - 1
    while t:
        n_steps += 1
        t >>= 1
    steps = []
    for step in range(n_steps):
        if not gather:
            dr = 1 << step
            to, frm = (me + n - dr) % n, (me + dr) % n
            n_sl = (n - 1 + (1 << step)) // (1 << (step + 1))
            delta = 1 << (step + 1)
            tx, rx = to, me
        else:
            dr = 1 << (n_steps - 1 - step)
            to, frm = (me + dr) % n, (me + n - dr) % n
            n_sl = (n - 1 + dr) // (1 << (n_steps - step))
            delta = 1 << (n_steps - step)
            tx, rx = me, (me - dr + n) % n
        txs, rxs = [], []
        for _ in range(n_sl):
            txs.append(tx)
            rxs.append(rx)
            tx = (tx + n - delta % n) % n
            rx = (rx + n - delta % n) % n
        steps.append((to, frm, txs, rxs))
    return steps


def nhr_reduce_scatter(dtype, op, work, bounds):
    """NHR reduce-scatter steps in place on per-rank working arrays: at each step the receiver's slice becomes
    sender_partial (src) (op) receiver_partial (dst) (write-reduce)."""
    n = len(work)
    per_rank = [nhr_steps(n, r, False) for r in range(n)]
    for step in range(len(per_rank[0])):
        old = [w.copy() for w in work]
        for r in range(n):
            _, frm, _, rxs = per_rank[r][step]
            for s_idx in rxs:
                b, e = bounds[s_idx]
                if e > b:
                    work[r][b:e] = apply(dtype, op, old[frm][b:e], old[r][b:e])


def nhr_all_gather(work, bounds):
    n = len(work)
    per_rank = [nhr_steps(n, r, True) for r in range(n)]
    for step in range(len(per_rank[0])):
        old = [w.copy() for w in work]
        for r in range(n):
            _, frm, _, rxs = per_rank[r][step]
            for s_idx in rxs:
                b, e = bounds[s_idx]
                if e > b:
                    work[r][b:e] = old[frm][b:e]


def allreduce_nhr(dtype, op, xs, ccl=None):
    """NHR AllReduce per executor loop (AICPU_TS: transport bound = ccl, scratch multiple 1), floor slicing."""
    ccl = ccl_bytes_from_env() if ccl is None else ccl
    n = len(xs)
    es = xs[0].itemsize
    outs = [np.empty_like(x) for x in xs]
    for off, cnt in ref_loops(xs[0].size, es, ccl, 1, ccl):
        work = [x[off:off + cnt].copy() for x in xs]
        bounds = floor_bounds(cnt, n)
        nhr_reduce_scatter(dtype, op, work, bounds)
        nhr_all_gather(work, bounds)
        for r in range(n):
            outs[r][off:off + cnt] = work[r]
    return outs


def reduce_nhr(dtype, op, xs, root, ccl=None):
    """NHR Reduce per executor loop (transport bound UB_MAX_DATA_SIZE, scratch multiple 1), ceil slicing; the root's
    result after the NHR all-gather."""
    ccl = ccl_bytes_from_env() if ccl is None else ccl
    n = len(xs)
    es = xs[0].itemsize
    out = np.empty_like(xs[0])
    for off, cnt in ref_loops(xs[0].size, es, UB_MAX_DATA_SIZE, 1, ccl):
        work = [x[off:off + cnt].copy() for x in xs]
        bounds = ceil_bounds(cnt, n)
        nhr_reduce_scatter(dtype, op, work, bounds)
        nhr_all_gather(work, bounds)
        out[off:off + cnt] = work[root]
    return out


def reduce_scatter_nhr(dtype, op, xs, rc):
    """NHR ReduceScatter: slices are the blocks (ins_temp_reduce_scatter_nhr.cc:278-397, 407-456)."""
    n = len(xs)
    work = [x[:n * rc].copy() for x in xs]
    bounds = [(i * rc, (i + 1) * rc) for i in range(n)]
    nhr_reduce_scatter(dtype, op, work, bounds)
    return [work[me][me * rc:(me + 1) * rc].copy() for me in range(n)]


def reduce_scatter_o1(dtype, op, xs, rc):
    n = len(xs)
    blk = lambda r, q: xs[r][q * rc:(q + 1) * rc]  # noqa: E731
    return [fold(dtype, op, [blk(me, me)] + [blk(q, me) for q in range(n) if q != me]) for me in range(n)]


def reduce_scatter_ring(dtype, op, xs, rc):
    """Part k of every block travels ring k; rank me at position v gets acc = x_{cyc[v+1]}, then (op) x_{cyc[v+2]}
    .. x_{cyc[v+n]} = its own block, the travelling partial being src."""
    n = len(xs)
    es = xs[0].itemsize
    rings = ring_table(n)[:ring_count(n, rc * n * es)]
    outs = [np.empty(rc, xs[0].dtype) for _ in range(n)]
    for k, (pb, pe) in enumerate(ring_parts(rc, len(rings), es)):
        if pe <= pb:
            continue
        cyc = rings[k]
        for v, me in enumerate(cyc):
            sl = slice(me * rc + pb, me * rc + pe)
            acc = xs[cyc[(v + 1) % n]][sl].copy()
            for j in range(2, n + 1):
                acc = apply(dtype, op, acc, xs[cyc[(v + j) % n]][sl])
            outs[me][pb:pe] = acc
    return outs


def reduce_scatter_v_o1(dtype, op, xs, counts, displs):
    """ReduceScatterV mesh (ins_temp_reduce_scatter_v_mesh_1D.cc:107-146): rank me copies its own block
    [displs[me], displs[me] + counts[me]) and folds every peer's copy of it in ascending rank order (O1)."""
    n = len(xs)
    outs = []
    for me in range(n):
        b, e = displs[me], displs[me] + counts[me]
        outs.append(fold(dtype, op, [xs[me][b:e]] + [xs[q][b:e] for q in range(n) if q != me]) if e > b
                    else np.empty(0, xs[0].dtype))
    return outs


def reduce_oneshot(dtype, op, xs, root):
    n = len(xs)
    return fold(dtype, op, [xs[root]] + [xs[q] for q in range(n) if q != root])


def reduce_twoshot(dtype, op, xs, root, ccl=None):
    """Two-shot Reduce per executor loop (transport bound UB_MAX_DATA_SIZE, scratch multiple n), balanced slicing;
    slice c is folded in order O1 with its owner c first (reduce_mesh_1D_two_shot.cc:209-249)."""
    ccl = ccl_bytes_from_env() if ccl is None else ccl
    n = len(xs)
    es = xs[0].itemsize
    out = np.empty_like(xs[0])
    for off, cnt in ref_loops(xs[0].size, es, UB_MAX_DATA_SIZE, n, ccl):
        for c, (b, e) in enumerate(balanced_bounds(cnt, n)):
            if e > b:
                b0, e0 = off + b, off + e
                out[b0:e0] = fold(dtype, op, [xs[c][b0:e0]] + [xs[q][b0:e0] for q in range(n) if q != c])
    return out


def tree_fold(dtype, op, blocks):
    """O4 (ins_temp_reduce_scatter_order_preserved_group.cc:305-399): while more than one block remains, M = the
    largest power of two below the count, block i >= M folds into block i % M as dst = src (op) dst."""
    blocks = [np.ascontiguousarray(b).copy() for b in blocks]
    remaining = len(blocks)
    while remaining > 1:
        m = 1
        while m * 2 < remaining:
            m *= 2
        for src in range(m, remaining):
            blocks[src % m] = apply(dtype, op, blocks[src], blocks[src % m])
        remaining = m
    return blocks[0]


def allreduce_tree(dtype, op, xs):
    n = len(xs)
    es = xs[0].itemsize
    out = np.empty_like(xs[0])
    for b, e in chunk_bounds(xs[0].size, n, es):
        if e > b:
            out[b:e] = tree_fold(dtype, op, [x[b:e] for x in xs])
    return [out.copy() for _ in xs]


def reduce_scatter_tree(dtype, op, xs, rc):
    n = len(xs)
    return [tree_fold(dtype, op, [x[me * rc:(me + 1) * rc] for x in xs]) for me in range(n)]


def o6_peers(n, t, j):
    """Senders into sub-slice j of owner t, step by step (nextNum = s + j + 1, skipping n)."""
    out = []
    for s in range(n - 1):
        x = s + j + 1
        if x >= n:
            x += 1
        out.append((t + x) % n)
    return out


def even_subslices(count, parts):
    """…mesh_chunk.cc:166-183: `parts` slices, the first count % parts one element longer."""
    base, big = divmod(count, parts)
    out, b = [], 0
    for i in range(parts):
        ln = base + (1 if i < big else 0)
        out.append((b, b + ln))
        b += ln
    return out


def rs_subslices(count, parts, es):
    """…meshchunk.cc:155-180: parts-1 slices of floor(bytes / parts) rounded down to 4 KiB, the rest last; the even
    split when that leaves nothing (or parts < 2)."""
    align = count * es // parts // 4096 * 4096
    if parts < 2 or align == 0:
        return even_subslices(count, parts)
    a = align // es
    return [(i * a, (i + 1) * a) for i in range(parts - 1)] + [((parts - 1) * a, count)]


def allreduce_meshchunk(dtype, op, xs, ccl=None):
    """MeshChunk AllReduce per executor loop (AICPU_TS bound = ccl, scratch multiple 2), chunks of ceil(cnt / n)
    elements (no 128-B alignment), O6 per sub-slice."""
    ccl = ccl_bytes_from_env() if ccl is None else ccl
    n = len(xs)
    es = xs[0].itemsize
    out = np.empty_like(xs[0])
    for off, cnt in ref_loops(xs[0].size, es, ccl, 2, ccl):
        for t, (b, e) in enumerate(ceil_bounds(cnt, n)):
            for j, (sb, se) in enumerate(even_subslices(e - b, n - 1)):
                if se > sb:
                    lo, hi = off + b + sb, off + b + se
                    out[lo:hi] = fold(dtype, op, [xs[t][lo:hi]] + [xs[q][lo:hi] for q in o6_peers(n, t, j)])
    return [out.copy() for _ in xs]


def reduce_scatter_meshchunk(dtype, op, xs, rc, ccl=None):
    """MeshChunk ReduceScatter per executor loop of min(ccl - 1 MiB, (ccl - 1 MiB) / (n-1)) over recvCount
    (ins_v2_reduce_scatter_sole_executor.cc:32,160-175), 4-KiB sub-slices, O6 per sub-slice."""
    ccl = ccl_bytes_from_env() if ccl is None else ccl
    n = len(xs)
    es = xs[0].itemsize
    tmp = ccl - (1 << 20) if ccl > (1 << 20) else ccl
    loop_bytes = min(tmp, tmp // (n - 1) // ALIGN * ALIGN)
    per = max(1, loop_bytes // es)
    outs = [np.empty(rc, xs[0].dtype) for _ in xs]
    for off in range(0, rc, per):
        cnt = min(per, rc - off)
        for t in range(n):
            for j, (sb, se) in enumerate(rs_subslices(cnt, n - 1, es)):
                if se > sb:
                    lo, hi = t * rc + off + sb, t * rc + off + se
                    outs[t][off + sb:off + se] = fold(
                        dtype, op, [xs[t][lo:hi]] + [xs[q][lo:hi] for q in o6_peers(n, t, j)])
    return outs


# ----------------------------------------------------------------------------------------- AIV engine

AIV_NOT_MATCHED, AIV_AR_ONESHOT, AIV_AR_TWOSHOT_LARGE, AIV_AR_TWOSHOT_SMALL, AIV_RS_BIGDATA, AIV_RS_LOCAL_TREE = range(6)
AIV_CORE_LIMIT = 48  # MAX_NUM_BLOCKS, aiv_defines.h:35


def aiv_select(op_type, n, count, es, dt64, prod, strict=False, ccl=None, core_limit=AIV_CORE_LIMIT, aiv_only=False):
    """SelectAivAlgo (all_reduce_auto_selector.cc:591-683, reduce_scatter_auto_selector.cc:537-600) and the variant
    the AIV kernels take for `core_limit` vector cores (aiv_temp_all_reduce_mesh_1D_twoshot.cc:88-100,
    aiv_all_reduce_mesh_1d_twoshot.h:330-346; aiv_temp_reduce_scatter_mesh_1D.cc:87-97, aiv_reduce_scatter_op.h:23-37).
    dt64: UINT64 or FP64 (the AIV path rejects them). aiv_only: OpExecuteConfig::AIV_ONLY, which drops the
    8 MiB x rankSize bound (all_reduce_auto_selector.cc:650-661). Returns (variant, groupSize)."""
    ccl = ccl_bytes_from_env() if ccl is None else ccl
    if op_type not in (0, 1) or strict or prod or dt64 or n < 2:
        return AIV_NOT_MATCHED, 1
    if op_type == 0:
        size = count * es
        if (not aiv_only and size >= (8 << 20) * n) or size > ccl * 16:
            return AIV_NOT_MATCHED, 1
        if size < ((128 << 10) if n <= 8 else (512 << 10)):
            return AIV_AR_ONESHOT, 1
        blocks = core_limit // (n + 1) * (n + 1) if core_limit >= n + 1 else core_limit
        if blocks >= 2 * n:
            return AIV_AR_TWOSHOT_LARGE, (blocks - n) // n
        return AIV_AR_TWOSHOT_SMALL, 1
    total = count * es * n
    if (not aiv_only and total >= (8 << 20) * n) or total > ccl * 16:
        return AIV_NOT_MATCHED, 1
    blocks = core_limit
    if count * es < (512 << 10):
        blocks = min(blocks, 2 * n)
    return (AIV_RS_BIGDATA if blocks > 2 * n else AIV_RS_LOCAL_TREE), 1


def allreduce_aiv(dtype, op, xs, variant, group, ccl=None):
    """AIV AllReduce. One-shot (aiv_all_reduce_mesh_1d_oneshot.h:33-48) and small-core two-shot (:224-271): out =
    x_0, then (op)= x_1 .. x_{n-1}, order O2. Large-core two-shot (:145-181) per executor loop of
    min(UB_MAX_DATA_SIZE, ccl / 4): the loop is split into group * n balanced slices (the first cnt % (group*n) one
    longer); rank c owns slices [c*group, (c+1)*group) and folds its own copy first, then the others ascending (O1)."""
    if variant in (AIV_AR_ONESHOT, AIV_AR_TWOSHOT_SMALL):
        return allreduce_o2(dtype, op, xs)
    assert variant == AIV_AR_TWOSHOT_LARGE
    ccl = ccl_bytes_from_env() if ccl is None else ccl
    n = len(xs)
    es = xs[0].itemsize
    out = np.empty_like(xs[0])
    for off, cnt in ref_loops(xs[0].size, es, UB_MAX_DATA_SIZE, 4, ccl):
        sl = balanced_bounds(cnt, group * n)
        for c in range(n):
            b, e = off + sl[c * group][0], off + sl[(c + 1) * group - 1][1]
            if e > b:
                out[b:e] = fold(dtype, op, [xs[c][b:e]] + [xs[q][b:e] for q in range(n) if q != c])
    return [out.copy() for _ in xs]


def reduce_scatter_aiv(dtype, op, xs, rc, variant):
    """AIV ReduceScatter: the big-data kernel folds rank 0's copy of the block, then ranks 1 .. n-1 (O2,
    aiv_reduce_scatter_mesh_1d_bigdata.h:85-101); the local tree folds the pow-2 tree over the ranks (O4,
    aiv_reduce_scatter_local_tree.h:138-172)."""
    n = len(xs)
    if variant == AIV_RS_LOCAL_TREE:
        return reduce_scatter_tree(dtype, op, xs, rc)
    assert variant == AIV_RS_BIGDATA
    return [fold(dtype, op, [x[me * rc:(me + 1) * rc] for x in xs]) for me in range(n)]


ALGO_ONESHOT, ALGO_TWOSHOT, ALGO_RING, ALGO_RHD, ALGO_NHR, ALGO_TREE, ALGO_IPC, ALGO_MESHCHUNK = 1, 2, 3, 4, 5, 6, 7, 8
ALGO_IPC_AUTO = 9


def expected(op_type, algo, dtype, op, xs, count, root=0):
    """Per-rank expected outputs (Reduce: only the root's entry is meaningful; others are None)."""
    if op_type == 0:
        return {ALGO_ONESHOT: allreduce_o1, ALGO_TWOSHOT: allreduce_o2, ALGO_RING: allreduce_ring,
                ALGO_RHD: allreduce_rhd, ALGO_NHR: allreduce_nhr, ALGO_TREE: allreduce_tree,
                ALGO_IPC: allreduce_o2, ALGO_MESHCHUNK: allreduce_meshchunk}[algo](dtype, op, xs)
    if op_type == 1:
        return {ALGO_ONESHOT: reduce_scatter_o1, ALGO_RING: reduce_scatter_ring, ALGO_NHR: reduce_scatter_nhr,
                ALGO_TREE: reduce_scatter_tree, ALGO_IPC: reduce_scatter_o1,
                ALGO_MESHCHUNK: reduce_scatter_meshchunk}[algo](dtype, op, xs, count)
    if op_type == 3:
        full = np.concatenate([x[:count] for x in xs])
        return [full.copy() for _ in xs]
    if op_type == 2:
        r = {ALGO_ONESHOT: reduce_oneshot, ALGO_TWOSHOT: reduce_twoshot, ALGO_NHR: reduce_nhr,
             ALGO_IPC: reduce_twoshot}[algo](dtype, op, xs, root)
        return [r if q == root else None for q in range(len(xs))]
    raise ValueError(op_type)
