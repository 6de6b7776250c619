"""A caller's own device-to-device copy right before the collective.

r03's stale operands were the loopback link's device-to-device hipMemcpyAsync followed by a fold on the same stream
(DESIGN.md §5b). The library's own copies are its copy kernel since r04; a caller's are not: torch's copy_ of a
contiguous same-type device tensor is a hipMemcpyAsync. Here every rank thread fills its sendBuf with torch copy_ on
the collective's stream, from its own thread, immediately before HcclAllReduce, so the collective's first fold reads
bytes that copy has just written: the one-shot (single-stream) program, the two-stream two-shot and MeshChunk, and the
one-sided kernel. Several rounds per case, each from zeroed inputs, every output bit-exact against the schedule's
order. tests/test_gpu_link_copy.py also runs the first case at the end of the r03 failing order (the allocation
history that reproduced the link-copy failure).
"""
import numpy as np
import pytest
import torch

import hccl_amd as H
from oracle import oracle as O
from tests import sched_ref as R
from tests._util import to_device, to_host
from tests.test_gpu_collectives import AR, run_ranks

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,count,algo,inplace", [
    (4, 4099, H.Algo.AUTO, False),                      # one-shot O1, single-stream program
    (4, (3 << 20) + 5, H.Algo.MESH_TWOSHOT, False),     # two-stream two-shot O2: the first fold on the reduce stream
    (8, (40 << 20) // 4 + 3, H.Algo.MESH_CHUNK, True),  # MeshChunk O6 in place
    (4, 70001, H.Algo.IPC, False),                      # the one-sided kernel reads sendBuf in its phase 0
])
def test_user_copy_then_allreduce(n, count, algo, inplace):
    comms = H.loopback_world(n)
    streams = [torch.cuda.Stream() for _ in range(n)]
    try:
        for c in comms:
            c.set_algo(algo)
        for rnd in range(3):
            xs = [O.random_operands(O.FP32, count, seed=8800 + 100 * rnd + r, edge=False) for r in range(n)]
            srcs = [to_device(O.FP32, x) for x in xs]
            sends = [torch.zeros_like(s) for s in srcs]
            recvs = sends if inplace else [torch.zeros_like(s) for s in srcs]
            torch.cuda.synchronize()

            def body(r):
                with torch.cuda.stream(streams[r]):
                    sends[r].copy_(srcs[r])  # a device-to-device hipMemcpyAsync on the collective's stream
                comms[r].all_reduce(sends[r], recvs[r], H.HcclReduceOp.SUM, streams[r])

            run_ranks(n, body)
            torch.cuda.synchronize()
            used = comms[0].last_algo
            fam = H.select_algo(AR, n, count * 4, False) if used == H.Algo.IPC else used
            want = R.expected(AR, fam, O.FP32, O.SUM, xs, count)
            for r in range(n):
                got = to_host(O.FP32, recvs[r])
                bad = np.nonzero(got.view(np.uint32) != want[r].view(np.uint32))[0]
                assert not len(bad), (f"round {rnd} rank {r} ({H.Algo(used).name}): {len(bad)} wrong, first "
                                      f"{bad[:4].tolist()}, got {got[bad[0]]!r} want {want[r][bad[0]]!r}")
    finally:
        torch.cuda.synchronize()
        for c in comms:
            c.destroy()
