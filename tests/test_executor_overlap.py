"""The executor's derived synchronisation overlaps the reduce with the transfers, shown on the
executor's own plan (HcclAmdExecutorPlan: the units Execute issues and the cross-stream waits it derives) replayed on a
two-stream timeline by tools/executor_overlap_model.py (link units at 76.8 GB/s per peer link, reduce units at
6 TB/s of HBM). Host logic only, no GPU: the loopback world's own timelines are host-bound and cannot show it."""
import pytest

import hccl_amd as H
from tools import executor_overlap_model as M

C3 = (4 << 30) // 4


@pytest.mark.parametrize("algo", [H.Algo.RING, H.Algo.MESH_CHUNK, H.Algo.MESH_TWOSHOT, H.Algo.RHD])
def test_c3_reduce_runs_under_the_links(algo):
    row = M.model(H.OpType.ALLREDUCE, algo, 8, C3, H.HcclDataType.FP32)
    assert row["algo"] == algo.name
    assert row["reduce_hidden_frac"] >= 0.95, row
    assert row["makespan_over_bound"] <= 1.01, row


@pytest.mark.parametrize("algo", [H.Algo.RING, H.Algo.MESH_CHUNK])
def test_c4_reduce_scatter_overlaps(algo):
    row = M.model(H.OpType.REDUCE_SCATTER, algo, 8, (2 << 30) // 2 // 8, H.HcclDataType.BFP16)
    assert row["reduce_hidden_frac"] >= 0.7, row
    assert row["makespan_over_bound"] <= 1.05, row


def test_plan_waits_are_needed():
    """Negative control: the same plan with every cross-stream wait dropped lets a reduce start before the group that
    fills its staging has ended (so the waits the executor derives are not decoration)."""
    es = 4
    ops, nops, _, _ = H.build_schedule(H.OpType.ALLREDUCE, H.Algo.MESH_TWOSHOT, 8, 0, C3, H.HcclDataType.FP32)
    units = H.executor_plan(ops, nops, es)
    assert any(u["wait"] >= 0 for u in units)
    for u in units:
        if u["wait"] >= 0:
            assert units[u["wait"]]["stream"] != u["stream"]  # waits are always cross-stream
    first_reduce = next(i for i, u in enumerate(units) if not u["comm"])
    assert units[first_reduce]["wait"] >= 0  # the first fold waits for the scatter that filled its slots
