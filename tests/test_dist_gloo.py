"""The N > 1 path across real processes, on CPU: world_size 2 and 4 with torch.distributed's gloo backend.

Each process builds ITS OWN rank's schedule with the product's generator (HcclAmdBuildSchedule, host-only code in
libhccl_amd.so) and executes it: SEND/RECV groups become gloo isend/irecv batches posted together (the semantics
of one RCCL group), REDUCE/COPY records are applied with the oracle's element rule. The result must equal the
closed-form association order on every rank. This checks that independently generated per-rank programs match
message for message across process boundaries, as they must over RCCL.
"""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _execute(prog, nops, bufs, dtype, op):
    import numpy as np  # noqa: F811

    from oracle import oracle as O

    i = 0
    while i < nops:
        o = prog[i]
        if o.kind in (2, 3):
            g = o.group
            reqs, recvs = [], []
            while i < nops and prog[i].kind in (2, 3) and prog[i].group == g:
                p = prog[i]
                if p.kind == 2:
                    t = torch.from_numpy(bufs[p.srcBuf[0]][p.srcOff[0]:p.srcOff[0] + p.count].copy())
                    reqs.append(dist.P2POp(dist.isend, t.view(torch.uint8), p.peer))
                else:
                    t = torch.empty(p.count * bufs[0].itemsize, dtype=torch.uint8)
                    reqs.append(dist.P2POp(dist.irecv, t, p.peer))
                    recvs.append((p, t))
                i += 1
            for w in dist.batch_isend_irecv(reqs):
                w.wait()
            for p, t in recvs:
                bufs[p.dstBuf][p.dstOff:p.dstOff + p.count] = t.numpy().view(bufs[0].dtype)
            continue
        if o.kind == 0:
            bufs[o.dstBuf][o.dstOff:o.dstOff + o.count] = bufs[o.srcBuf[0]][o.srcOff[0]:o.srcOff[0] + o.count]
        else:
            srcs = [np.ascontiguousarray(bufs[o.srcBuf[j]][o.srcOff[j]:o.srcOff[j] + o.count]) for j in range(o.nsrc)]
            bufs[o.dstBuf][o.dstOff:o.dstOff + o.count] = O.reduce_n(dtype, op, srcs)
        i += 1


def _worker(rank, world, port, cases, q):
    import sys
    sys.path.insert(0, ROOT)
    try:
        import hccl_amd as H
        from oracle import oracle as O
        from tests import sched_ref as R

        import datetime
        store = dist.TCPStore("127.0.0.1", port, is_master=False, timeout=datetime.timedelta(seconds=120))
        dist.init_process_group("gloo", store=store, rank=rank, world_size=world)
        for op_type, algo, count, dtype, op in cases:
            prog, nops, used, scratch = H.build_schedule(op_type, algo, world, rank, count, dtype, root=world - 1,
                                                         piece_bytes=4096)
            in_count = count * world if op_type == 1 else count
            xs = [O.random_operands(dtype, in_count, seed=1234 + r, edge=False, small_ints=True)
                  for r in range(world)]
            st = O.NP_STORAGE[dtype]
            bufs = [xs[rank].copy(), np.zeros(count, st), np.zeros(max(scratch, 1), st)]
            _execute(prog, nops, bufs, dtype, op)
            want = R.expected(op_type, used, dtype, op, xs, count, root=world - 1)[rank]
            if want is not None and not O.equal_bits(dtype, bufs[1], want):
                raise AssertionError(f"rank {rank} case {(op_type, algo, count, dtype, op)} mismatch")
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, f"{type(e).__name__}: {e}\n{traceback.format_exc()}"))


def _launch(world, cases):
    import datetime
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    # the store's server lives in this process on a port the OS picks: no free-port race with parallel test workers
    master = dist.TCPStore("127.0.0.1", 0, is_master=True, wait_for_workers=False,
                           timeout=datetime.timedelta(seconds=120))
    port = master.port
    procs = [ctx.Process(target=_worker, args=(r, world, port, cases, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    bad = [r for r in res if r[1] != "ok"]
    assert not bad, bad


FP32, FP16, INT32, SUM, MAX = 4, 3, 2, 0, 2


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_allreduce_reducescatter_reduce(world):
    cases = [
        (0, 1, 3001, FP32, SUM), (0, 2, 5003, FP32, SUM), (0, 3, 5003, FP32, SUM), (0, 4, 5003, FP32, SUM),
        (0, 5, 5003, FP32, SUM), (0, 6, 5003, FP32, SUM), (0, 8, 5003, FP32, SUM),
        (0, 2, 2049, FP16, MAX), (1, 1, 1537, FP32, SUM), (1, 3, 1537, INT32, SUM), (1, 8, 1537, FP32, SUM),
        (2, 1, 4097, FP32, SUM), (2, 2, 4097, FP32, SUM),
    ]
    _launch(world, cases)


def test_gloo_eight_ranks_every_link_schedules():
    """World 8 (the driver's N = 8 shape): the 7-ring and 7-instance RHD schedules (every link in every step), MeshChunk
    (C3 / C4 selection) and the two-shot, each rank generating its own program."""
    cases = [(0, 3, 20011, FP32, SUM), (0, 4, 20011, FP32, SUM), (0, 8, 20011, FP32, SUM), (0, 2, 20011, FP32, SUM),
             (1, 3, 2503, FP32, SUM), (1, 8, 2503, FP16, SUM)]
    _launch(8, cases)
