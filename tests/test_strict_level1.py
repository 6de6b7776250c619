"""HCCL_DETERMINISTIC=strict at n <= 8, pinned where the bits come from.

At n <= MAX_RANK_NUM_FOR_ORDER_PRESERVED (8, common/order_preserved_common.h:22) the reference selects
AicpuReduceScatterStrictOrderedMesh (reduce_scatter_auto_selector.cc:406-413) and AicpuAllReduceStrictOrderedMesh
(all_reduce_auto_selector.cc:412-418), whose reduce step is InsTempReduceScatterOrderPreservedLevel1
(ins_v2_reduce_scatter_order_preserved_executor.cc:233-235; the AllReduce's RS half,
ins_v2_all_reduce_order_preserved_executor.cc:449-451). This file restates that template literally:
  * CalcOutputIndex(round, localRank) = (round + localRank) % n (…order_preserved_level1.cc:176-181);
  * PreLocalCopy: receiver t's own block goes to CCL slot CalcOutputIndex(t, t) (:196-215);
  * RunAllToAll: sender s writes receiver t's block into t's CCL slot CalcOutputIndex(t, s) (:219-296, txOutputIndex
    = CalcOutputIndex(nextRank, myAlgRank) at :274-278);
  * RunLocalReduce: blocks at virtual index v >= M fold into v % M, M the largest power of two below the remaining
    count, repeated; virtual index v reads slot CalcOutputIndex(v, t) (:322-400); the result is at virtual index 0.
It then checks (1) that virtual index v always holds source rank v's data (so the tree is over source ranks, the same
on every receiver), and (2) that the restatement, run on random fp32 data in float32, gives the bits of this build's
ORDER_PRESERVED schedule replayed by the oracle (schedule.cc), for ReduceScatter and AllReduce at 3..8 ranks.
Host only: no GPU.
"""
import numpy as np
import pytest

import hccl_amd as H
from oracle import oracle as O

RS, AR = 1, 0
STRICT = 6  # HCCL_AMD_ALGO_ORDER_PRESERVED


def calc_output_index(rnd, local_rank, n):  # …order_preserved_level1.cc:176-181
    return (rnd + local_rank) % n


def largest_pow2_below(v):  # GetLargestPowerOf2LessThan, :300-310
    if v <= 1:
        return 0
    p = 1
    while p * 2 < v:
        p *= 2
    return p


def level1_receiver(t, blocks_for_t, n):
    """Receiver t (myAlgRank) of the Level1 template. blocks_for_t[s] = source s's block for t. Returns the reduced
    block and, per CCL slot, which source wrote it."""
    ccl, writer = [None] * n, [None] * n
    k = calc_output_index(t, t, n)  # PreLocalCopy
    ccl[k], writer[k] = blocks_for_t[t].copy(), t
    for s in range(n):  # RunAllToAll on every other rank s: nextRank = t for rankIdx = (t - s) mod n
        if s == t:
            continue
        k = calc_output_index(t, s, n)
        assert ccl[k] is None, "two writers into one slot"
        ccl[k], writer[k] = blocks_for_t[s].copy(), s
    for v in range(n):  # the tree's virtual index v is source rank v on every receiver
        assert writer[calc_output_index(v, t, n)] == v
    rem = n
    while rem > 1:  # RunLocalReduce
        m = largest_pow2_below(rem)
        for v in range(m, rem):
            src = ccl[calc_output_index(v, t, n)]
            dst = ccl[calc_output_index(v % m, t, n)]
            dst[:] = src + dst  # LocalReduce(src, dst): dst = src (+) dst in float32 (AicpuReduceTemplate :1327)
        rem = m
    return ccl[calc_output_index(0, t, n)]


def replay(op_type, n, count, xs):
    progs, scratch = [], 0
    for r in range(n):
        arr, nops, used, se = H.build_schedule(op_type, STRICT, n, r, count, O.FP32)
        assert used == STRICT
        progs.append((arr, nops))
        scratch = max(scratch, se)
    out_count = count
    bufs = [[x.copy(), np.zeros(out_count, np.float32), np.zeros(max(scratch, 1), np.float32)] for x in xs]
    assert O.replay(n, O.FP32, O.SUM, progs, bufs) == 0
    return [b[1] for b in bufs]


@pytest.mark.parametrize("n", [3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("count", [1, 37, 4099])
def test_level1_reduce_scatter_is_the_strict_schedule(n, count):
    rng = np.random.default_rng(1000 * n + count)
    xs = [rng.standard_normal(n * count).astype(np.float32) for _ in range(n)]
    want = replay(RS, n, count, xs)
    for t in range(n):
        got = level1_receiver(t, [xs[s][t * count:(t + 1) * count] for s in range(n)], n)
        assert np.array_equal(got.view(np.uint32), want[t].view(np.uint32)), t


@pytest.mark.parametrize("n", [3, 4, 5, 6, 7, 8])
def test_level1_allreduce_is_slicing_independent_and_the_strict_schedule(n):
    """The AllReduce's RS half is the same template over the executor's per-rank slices; the tree is over source ranks,
    so the value of an element does not depend on which owner's slice it is in: the elementwise tree gives the bits for
    any slicing, and equals the schedule's replay."""
    count = 10007
    rng = np.random.default_rng(77 + n)
    xs = [rng.standard_normal(count).astype(np.float32) for _ in range(n)]
    want = replay(AR, n, count, xs)
    tree = level1_receiver(0, [x.copy() for x in xs], n)  # the whole vector as one block (any slicing)
    # two other slicings: the reference executor's (floor, tail on the last rank) and a ragged one
    for cuts in (np.linspace(0, count, n + 1).astype(int), np.array([0] + sorted(rng.choice(count, n - 1)) + [count])):
        parts = [level1_receiver(t, [x[cuts[t]:cuts[t + 1]] for x in xs], n) for t in range(n)]
        assert np.array_equal(np.concatenate(parts).view(np.uint32), tree.view(np.uint32))
    for r in range(n):
        assert np.array_equal(want[r].view(np.uint32), tree.view(np.uint32)), r
    # and the order matters on this data: the plain rank-order left fold differs somewhere
    acc = xs[0].copy()
    for x in xs[1:]:
        acc = x + acc
    assert not np.array_equal(acc.view(np.uint32), tree.view(np.uint32))
