"""The AIV engine's selection (HcclAmdSelectAivAlgo) against an independent restatement of SelectAivAlgo and the AIV
kernels' variant split (tests/sched_ref.py aiv_select): every op type, rank count, size edge, dtype, op, core limit
and the STRICT mode. Host logic only, no GPU."""
import itertools

import pytest

import hccl_amd as H
from oracle import oracle as O
from tests import sched_ref as R

ES = {O.INT8: 1, O.INT16: 2, O.INT32: 4, O.INT64: 8, O.UINT64: 8, O.FP16: 2, O.BFP16: 2, O.FP32: 4, O.FP64: 8}


def _counts(es, n):
    edges = [1, (128 << 10) // es - 1, (128 << 10) // es, (512 << 10) // es - 1, (512 << 10) // es,
             (8 << 20) * n // es - 1, (8 << 20) * n // es, (8 << 20) // es, 12345]
    edges += [(200 << 20) * 16 // es, (200 << 20) * 16 // es + 1]  # the 16 CCL buffers bound (AIV_ONLY reaches it)
    return sorted({max(1, c) for c in edges})


@pytest.mark.parametrize("n", [2, 3, 4, 8, 9, 16])
@pytest.mark.parametrize("core_limit", [48, 56, 16, 9, 4])
def test_aiv_selection_matches_restatement(n, core_limit):
    for op_type, dt, op, strict, only in itertools.product((0, 1, 2), ES, O.OPS, (False, True), (False, True)):
        es = ES[dt]
        for count in _counts(es, n):
            got, group = H.select_aiv_algo(op_type, n, count, dt, op, core_limit, strict, only)
            want, wgroup = R.aiv_select(op_type, n, count, es, dt in (O.UINT64, O.FP64), op == O.PROD, strict,
                                        ccl=R.ccl_bytes_from_env(), core_limit=core_limit, aiv_only=only)
            assert (int(got), group) == (want, wgroup), (op_type, n, count, dt, op, strict, only, core_limit)


def test_aiv_default_core_limit_variants_at_eight_ranks():
    """With 48 vector cores and 8 ranks: one-shot below 128 KiB, the large-core two-shot (4 slices per rank) up to
    64 MiB, then the AICPU engine; ReduceScatter takes the local tree below 512 KiB of output, big-data above."""
    sel = lambda t, c, dt=O.FP32: H.select_aiv_algo(t, 8, c, dt, O.SUM)  # noqa: E731
    assert sel(0, 1024) == (H.AivVariant.AR_ONESHOT, 1)
    assert sel(0, (128 << 10) // 4) == (H.AivVariant.AR_TWOSHOT_LARGE, 4)
    assert sel(0, (64 << 20) // 4 - 1) == (H.AivVariant.AR_TWOSHOT_LARGE, 4)
    assert sel(0, (64 << 20) // 4)[0] == H.AivVariant.NOT_MATCHED
    assert sel(1, 1000)[0] == H.AivVariant.RS_LOCAL_TREE
    assert sel(1, (512 << 10) // 4)[0] == H.AivVariant.RS_BIGDATA
    assert sel(2, 1000)[0] == H.AivVariant.NOT_MATCHED  # Reduce has no AIV selection
    assert sel(0, 1000, O.FP64)[0] == H.AivVariant.NOT_MATCHED


def test_aiv_only_lifts_the_per_rank_bound():
    """AIV_ONLY keeps the AIV engine above 8 MiB x n (up to 16 CCL buffers); what it still does not match is an error
    at the entry (HCCL_E_NOT_SUPPORT), not a fallback."""
    sel = lambda t, c, dt=O.FP32: H.select_aiv_algo(t, 8, c, dt, O.SUM, aiv_only=True)  # noqa: E731
    assert sel(0, (64 << 20) // 4) == (H.AivVariant.AR_TWOSHOT_LARGE, 4)
    assert sel(0, (200 << 20) * 16 // 4) == (H.AivVariant.AR_TWOSHOT_LARGE, 4)
    assert sel(0, (200 << 20) * 16 // 4 + 1)[0] == H.AivVariant.NOT_MATCHED
    assert sel(1, (64 << 20) // 4)[0] == H.AivVariant.RS_BIGDATA
    assert H.Algo.AIV_ONLY == 11
