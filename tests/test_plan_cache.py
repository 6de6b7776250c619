"""The compiled-collective cache (executor.cc CompileCollective) reuses an executor plan for every call whose buffers
overlap the same way. That rests on a property of PlanUnits checked here on the executor's own plans (host only):
the plan is unchanged when the buffers move while keeping their overlap relation (disjoint buffers anywhere, in order
or not; in-place buffers at any common address), and it can change when the relation changes (in-place vs
out-of-place), which is why the relation is part of the cache key."""
import pytest

import hccl_amd as H

AR, RS, RED = H.OpType.ALLREDUCE, H.OpType.REDUCE_SCATTER, H.OpType.REDUCE
T = 1 << 40

CASES = [(AR, H.Algo.MESH_TWOSHOT, 8, (64 << 20) // 4 + 3), (AR, H.Algo.RING, 8, (64 << 20) // 4 + 3),
         (AR, H.Algo.RHD, 8, (32 << 20) // 4), (AR, H.Algo.NHR, 5, (16 << 20) // 4 + 1),
         (AR, H.Algo.MESH_CHUNK, 8, (300 << 20) // 4 + 7), (AR, H.Algo.MESH_ONESHOT, 4, (4 << 20) // 4),
         (AR, H.Algo.ORDER_PRESERVED, 6, (8 << 20) // 4 + 5), (RS, H.Algo.MESH_CHUNK, 8, (16 << 20) // 4),
         (RS, H.Algo.RING, 8, (16 << 20) // 4 + 1), (RS, H.Algo.MESH_ONESHOT, 3, (8 << 20) // 4),
         (RED, H.Algo.MESH_TWOSHOT, 4, (16 << 20) // 4 + 2), (RED, H.Algo.MESH_ONESHOT, 4, (2 << 20) // 4)]


def plan(op_type, algo, n, rank, count, bases):
    ops, nops, _, _ = H.build_schedule(op_type, algo, n, rank, count, H.HcclDataType.FP32)
    return H.executor_plan(ops, nops, 4, bases)


@pytest.mark.parametrize("op_type,algo,n,count", CASES)
@pytest.mark.parametrize("rank", [0, 1])
def test_plan_is_translation_invariant(op_type, algo, n, rank, count):
    disjoint = [(1 * T, 2 * T, 3 * T), (5 * T + 4096, T // 2, 7 * T + 128), (9 * T, 3 * T + 256, T)]
    ref = plan(op_type, algo, n, rank, count, disjoint[0])
    for b in disjoint[1:]:
        assert plan(op_type, algo, n, rank, count, b) == ref, b
    if op_type != RS:  # in-place: ReduceScatter's recvBuf is a block of sendBuf, not the same base
        inref = plan(op_type, algo, n, rank, count, (2 * T, 2 * T, 5 * T))
        for b in [(7 * T + 512, 7 * T + 512, T), (T // 4, T // 4, 3 * T)]:
            assert plan(op_type, algo, n, rank, count, b) == inref, b


def test_relation_is_part_of_the_key():
    """The plan does depend on the relation: a send of sendBuf followed by a fold into recvBuf needs no wait when the
    buffers are disjoint and a write-after-read wait when they are the same buffer (in-place)."""
    ops = (H.HcclAmdIrOp * 2)()
    ops[0].kind, ops[0].peer, ops[0].nsrc, ops[0].group, ops[0].count = H.IrKind.SEND, 1, 1, 0, 1024
    ops[0].dstBuf, ops[0].srcBuf[0], ops[0].srcOff[0] = -1, 0, 0
    ops[1].kind, ops[1].peer, ops[1].nsrc, ops[1].count = H.IrKind.REDUCE, -1, 2, 1024
    ops[1].dstBuf, ops[1].dstOff = 1, 0
    ops[1].srcBuf[0], ops[1].srcOff[0], ops[1].srcBuf[1], ops[1].srcOff[1] = 2, 0, 2, 1024
    out = H.executor_plan(ops, 2, 4, (T, 2 * T, 3 * T))
    inp = H.executor_plan(ops, 2, 4, (T, T, 3 * T))
    assert out[1]["wait"] == -1
    assert inp[1]["wait"] == 0
