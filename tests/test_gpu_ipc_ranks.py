"""The one-sided IPC AllReduce in RANK mode: n separate processes, each one rank with its own launch, peers' staging
and flags opened from hipIpcMemHandles — the path the 8-GPU node runs (here all ranks share the one GPU, which the
bootstrap-only communicator of HcclAmdCommInitHostExchange allows; RCCL refuses two ranks on one device).
Expected results: order O2 (acc = x_0, then x_1 .. x_{n-1}; ins_temp_all_reduce_mesh_1D_two_shot.cc:327-335), from
the oracle's fold, bit-exact."""
import datetime
import multiprocessing as mp
import os
import socket
import time
import traceback

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

AR, RS, RED, AG = 0, 1, 2, 3
# (collective, dtype, op, count): ragged counts, every reduce dtype family, counts that need several pieces per chunk
CASES = [
    (AR, O.FP32, O.SUM, 1), (AR, O.FP32, O.SUM, 4099), (AR, O.FP32, O.MAX, 100003), (AR, O.FP32, O.SUM, (36 << 20) + 11),
    (AR, O.FP16, O.SUM, 65537), (AR, O.BFP16, O.SUM, 70001), (AR, O.BFP16, O.MIN, 4097), (AR, O.INT32, O.PROD, 9999),
    (AR, O.INT8, O.SUM, 33333), (AR, O.INT64, O.MAX, 5000), (AR, O.FP64, O.SUM, 12345), (AR, O.FP32, O.PROD, 777),
    (RS, O.FP32, O.SUM, 3), (RS, O.FP32, O.SUM, 50001), (RS, O.BFP16, O.MAX, 20003), (RS, O.FP32, O.SUM, (17 << 20) + 5),
    (RED, O.FP32, O.SUM, 5), (RED, O.FP16, O.SUM, 60001), (RED, O.FP32, O.MIN, (36 << 20) + 7),
    (AR, O.FP32, O.SUM, 250001),
    # HCCL_AMD_ALGO_IPC (9): the order family the auto selector picks, so the auto path's bits over IPC:
    # one-shot O1 AllReduce / Reduce, MeshChunk O6 (AllReduce above 16 MiB at n = 2, ReduceScatter above 4 MiB at
    # n = 4 and 1 MiB at n = 2), two-shot O2 AllReduce at n = 4
    (AR, O.FP32, O.SUM, 5001, 9), (AR, O.FP32, O.SUM, (20 << 20) // 4 + 3, 9), (RS, O.FP32, O.SUM, (5 << 20) // 4 + 1, 9),
    (RED, O.FP16, O.SUM, 3001, 9), (AR, O.BFP16, O.MAX, 70001, 9),
    # HcclAmdCommSetIpcBlocks: 256 and 64 workgroups per launch instead of 128 (different windows per block)
    (AR, O.FP32, O.SUM, (20 << 20) // 4 + 3, 9, 256), (AR, O.FP32, O.SUM, 40961, 7, 64),
    (RS, O.FP32, O.SUM, 70001, 7, 256),
    # AllGather (data movement, one barrier per round): ragged, several rounds, and between reducing calls
    (AG, O.FP16, O.SUM, 33333, 9), (AG, O.FP32, O.SUM, (20 << 20) + 3, 9), (AG, O.INT8, O.SUM, 5, 9),
    (AR, O.FP32, O.SUM, 4099, 9),
    # HCCL_AMD_ALGO_AIV (10): the AIV engine's variants (default 48 vector cores): one-shot O2, large-core two-shot
    # O1 over balanced groups (ragged: chunk starts off the vector grid), ReduceScatter local tree O4 and big-data O2
    (AR, O.FP32, O.SUM, 5001, 10), (AR, O.FP32, O.SUM, (1 << 20) + 3, 10), (AR, O.BFP16, O.MAX, 300001, 10),
    (RS, O.FP32, O.SUM, 1001, 10), (RS, O.FP16, O.SUM, (1 << 18) + 5, 10), (AR, O.FP32, O.SUM, 4099, 9),
]
UNALIGNED_CASE = CASES.index((AR, O.FP32, O.SUM, 250001))
ROOT = 1


def _in_count(kind, count, n):
    return count * n if kind == RS else count


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs(dtype, count, n, seed):
    return [O.random_operands(dtype, count, seed * 1000 + r) for r in range(n)]


def _rank_main(rank, n, port, q, fence=None):
    os.environ["HCCL_AMD_IPC_TIMEOUT_MS"] = "20000"  # a lost peer shows as a status bit, never a hang
    if fence is not None:
        os.environ["HCCL_AMD_IPC_LIGHT_FENCE"] = fence
    os.makedirs("gpurun_out", exist_ok=True)
    progress = open(f"gpurun_out/ipc_ranks_n{n}_r{rank}.log", "w", buffering=1)
    try:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=n,
                                timeout=datetime.timedelta(seconds=120))
        torch.cuda.set_device(0)
        import hccl_amd as H
        import sched_ref as R
        from _util import to_device, to_host

        def all_gather(b):
            out = [None] * n
            dist.all_gather_object(out, b)
            return out

        comm = H.comm_init_host_exchange(n, rank, all_gather)
        stream = torch.cuda.Stream()
        results = []
        for i, case in enumerate(CASES):
            kind, dtype, op, count = case[:4]
            forced = case[4] if len(case) > 4 else None
            comm.set_algo(forced if forced is not None else R.ALGO_IPC)
            comm.set_ipc_blocks(case[5] if len(case) > 5 else 0)
            progress.write(f"case {i} {CASES[i]} start\n")
            send = to_device(dtype, _inputs(dtype, _in_count(kind, count, n), n, i)[rank])
            recv = torch.zeros(count * n if kind == AG else count, dtype=send.dtype, device=send.device)
            if i == UNALIGNED_CASE and rank == n - 1:  # one rank with unaligned buffers: still the IPC path
                send = torch.cat([send[:1], send])[1:]
                recv = torch.empty(count + 1, dtype=send.dtype, device=send.device)[1:]
            torch.cuda.synchronize()
            if kind == AR:
                comm.all_reduce(send, recv, op, stream=stream)
            elif kind == RS:
                comm.reduce_scatter(send, recv, op, stream=stream)
            elif kind == AG:
                comm.all_gather(send, recv, stream=stream)
            else:
                comm.reduce(send, recv, ROOT % n, op, stream=stream)
            stream.synchronize()
            status = comm.ipc_status()
            got = to_host(dtype, recv)
            ok = True
            if kind == AG:
                want = np.concatenate(_inputs(dtype, count, n, i))
                ok = O.equal_bits(dtype, got, want)
            elif not (kind == RED and rank != ROOT % n):
                xs = _inputs(dtype, _in_count(kind, count, n), n, i)
                fam = R.ALGO_IPC
                if forced == 9:
                    special = dtype in (O.INT64, O.UINT64, O.FP64) or op == O.PROD
                    nbytes = count * O.NP_STORAGE[dtype]().itemsize
                    fam = H.select_algo(kind, n, nbytes, special)
                if forced == 10:
                    es = O.NP_STORAGE[dtype]().itemsize
                    variant, group = R.aiv_select(kind, n, count, es, dtype in (O.UINT64, O.FP64), op == O.PROD)
                    want = (R.allreduce_aiv(dtype, op, xs, variant, group) if kind == AR
                            else R.reduce_scatter_aiv(dtype, op, xs, count, variant))[rank]
                else:
                    want = R.expected(kind, fam, dtype, op, xs, count, root=ROOT % n)[rank]
                ok = O.equal_bits(dtype, got, want)
            progress.write(f"case {i} done status {status} algo {comm.last_algo} ok {ok}\n")
            results.append((i, status, comm.last_algo, ok))
            if max(all_gather(status & 1)) != 0:  # every rank stops together after a barrier timeout anywhere
                break
        # HIP graph: AllReduce (three sizes: the LL one-shot, a staged one-shot, two-shot), ReduceScatter (staged and
        # LL) and AllGather captured once,
        # then replayed with fresh inputs. The barrier epochs live on the device, so each replay takes new ones as a
        # new call would. Small integers in fp32: every order gives the same bits.
        comm.set_algo(R.ALGO_IPC)
        comm.set_ipc_blocks(0)
        sizes = (1000, 300001, (3 << 20) + 5)
        ar_in = [torch.zeros(c, device="cuda") for c in sizes]
        ar_out = [torch.zeros(c, device="cuda") for c in sizes]
        rs_len, ag_len, rs_small = 70001, 50003, 1001  # rs_small: the LL ReduceScatter (blocks under 64 KiB)
        rs_in = torch.zeros(n * rs_len, device="cuda")
        rs_out = torch.zeros(rs_len, device="cuda")
        rss_in = torch.zeros(n * rs_small, device="cuda")
        rss_out = torch.zeros(rs_small, device="cuda")
        ag_in = torch.zeros(ag_len, device="cuda")
        ag_out = torch.zeros(n * ag_len, device="cuda")
        ramp = torch.arange(n * rs_len, device="cuda", dtype=torch.float32) % 97
        graph = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        with torch.cuda.graph(graph, stream=torch.cuda.Stream()):
            cs = torch.cuda.current_stream()
            for x, y in zip(ar_in, ar_out):
                comm.all_reduce(x, y, O.SUM, stream=cs)
            comm.reduce_scatter(rs_in, rs_out, O.SUM, stream=cs)
            comm.reduce_scatter(rss_in, rss_out, O.SUM, stream=cs)
            comm.all_gather(ag_in, ag_out, stream=cs)
        graph_ok = []
        for rep in range(4):
            v = float((rank + 1) * (rep + 1))
            for x in ar_in:
                x.fill_(v)
            rs_in.copy_(ramp + v)
            rss_in.copy_(ramp[:n * rs_small] + v)
            ag_in.fill_(v)
            torch.cuda.synchronize()
            graph.replay()
            torch.cuda.synchronize()
            tot = float((rep + 1) * n * (n + 1) // 2)
            ok = all(bool(torch.all(y == tot).item()) for y in ar_out)
            ok = ok and bool(torch.all(rs_out == n * ramp[rank * rs_len:(rank + 1) * rs_len] + tot).item())
            ok = ok and bool(torch.all(rss_out == n * ramp[rank * rs_small:(rank + 1) * rs_small] + tot).item())
            want = torch.cat([torch.full((ag_len,), float((q + 1) * (rep + 1)), device="cuda") for q in range(n)])
            ok = ok and bool(torch.equal(ag_out, want))
            graph_ok.append(ok)
            progress.write(f"graph replay {rep} ok {ok}\n")
        results.append(("graph", graph_ok, comm.ipc_status() & 1))
        dist.barrier()
        comm.destroy()  # collective: no rank unmaps while a peer's kernel may still store into it
        progress.write("destroyed\n")
        dist.destroy_process_group()
        q.put((rank, "ok", results))
    except Exception:  # noqa: BLE001
        progress.write(traceback.format_exc())
        q.put((rank, traceback.format_exc(), None))
        time.sleep(10)  # peers' kernels are bounded: let them drain before this process's memory goes away


@pytest.mark.parametrize("n,fence", [(2, None), (4, None), (2, "1")])
def test_ipc_collectives_rank_mode(n, fence):
    """Rank mode with its default system-scope barrier fences, and once (n = 2) with the light fences forced
    (HCCL_AMD_IPC_LIGHT_FENCE=1, the loopback world's default)."""
    import sched_ref as R
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, n, port, q, fence)) for r in range(n)]
    for p in procs:
        p.start()
    try:
        got = {}
        for _ in procs:
            rank, msg, res = q.get(timeout=300)
            got[rank] = (msg, res)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(n):
        assert got[r][0] == "ok", f"rank {r}:\n{got[r][0]}"
    for r in range(n):
        assert got[r][1][-1] == ("graph", [True] * 4, 0), got[r][1][-1]  # every replay right, no barrier timeout
        got[r] = (got[r][0], got[r][1][:-1])
    for r in range(n):
        assert len(got[r][1]) == len(CASES), f"rank {r} stopped after case {len(got[r][1]) - 1}"
        for i, status, algo, _ok in got[r][1]:
            assert status & 1 == 0, f"rank {r} case {CASES[i]}: barrier timeout (status {status:#x})"
            assert algo == (CASES[i][4] if len(CASES[i]) > 4 else R.ALGO_IPC)
    for r in range(n):
        for i, status, algo, ok in got[r][1]:
            assert ok, f"rank {r} case {CASES[i]} differs from the reference order"


def _lost_peer_main(rank, port, q, count=1 << 20):
    # the bound comes from the reference's own variable (AIV-mode rule: seconds, two decimals)
    os.environ.pop("HCCL_AMD_IPC_TIMEOUT_MS", None)
    os.environ["HCCL_EXEC_TIMEOUT"] = "1.5"
    os.makedirs("gpurun_out", exist_ok=True)
    progress = open(f"gpurun_out/ipc_lost_peer_r{rank}.log", "w", buffering=1)
    try:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2,
                                timeout=datetime.timedelta(seconds=120))
        torch.cuda.set_device(0)
        import hccl_amd as H

        def all_gather(b):
            out = [None] * 2
            dist.all_gather_object(out, b)
            return out

        def code_of(fn):
            try:
                fn()
                return 0
            except H.HcclError as e:
                return e.code

        comm = H.comm_init_host_exchange(2, rank, all_gather)
        comm.set_algo(H.Algo.IPC)  # the auto family's one-shot: the LL form at the small size
        stream = torch.cuda.Stream()
        x = torch.full((count,), float(rank + 1), device="cuda")
        y = torch.empty_like(x)
        torch.cuda.synchronize()
        comm.all_reduce(x, y, H.HcclReduceOp.SUM, stream=stream)  # both ranks: set-up + a good call
        stream.synchronize()
        res = {"first_status": comm.ipc_status(), "first_ok": bool(torch.all(y == 3.0).item()),
               "first_async": comm.async_error(), "timeout_ms": H.lib.HcclAmdIpcTimeoutMs(),
               "ll_launches": comm.ipc_ll_launches()}
        progress.write(f"first {res}\n")
        dist.barrier()
        if rank == 0:  # rank 1 never joins this call
            t0 = time.time()
            comm.all_reduce(x, y, H.HcclReduceOp.SUM, stream=stream)  # enqueued: returns before the wait
            res["lost_rc"] = 0
            stream.synchronize()
            res["lost_s"] = time.time() - t0
            res["lost_status"] = comm.ipc_status()
            res["async_after_lost"] = comm.async_error()
            # the next entry observes the failure and returns it; every later one finds the communicator failed
            t0 = time.time()
            res["next_rc"] = code_of(lambda: comm.all_reduce(x, y, H.HcclReduceOp.SUM, stream=stream))
            res["then_rc"] = code_of(lambda: comm.all_reduce(x, y, H.HcclReduceOp.SUM, stream=stream))
            res["rs_rc"] = code_of(lambda: comm.reduce_scatter(x, y[: x.numel() // 2], H.HcclReduceOp.SUM,
                                                              stream=stream))
            stream.synchronize()
            res["after_s"] = time.time() - t0
            res["async_later"] = comm.async_error()
            progress.write(f"lost {res}\n")
        dist.barrier()
        comm.destroy()
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception:  # noqa: BLE001
        progress.write(traceback.format_exc())
        q.put((rank, traceback.format_exc(), None))
        time.sleep(10)


@pytest.mark.parametrize("count", [1 << 20, 256], ids=["staged", "ll"])
def test_ipc_lost_peer_fails_the_communicator(count):
    """A peer that never joins: the wait (staged: the barrier; LL: the flag poll) gives up after HCCL_EXEC_TIMEOUT (no
    hang); the next collective returns
    HCCL_E_TIMEOUT, every later one HCCL_E_SUSPENDING (the reference's status gate, op_common.cc:89-97), and
    HcclGetCommAsyncError reports HCCL_E_TIMEOUT without a device synchronisation; teardown still completes."""
    import hccl_amd as H
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_lost_peer_main, args=(r, port, q, count)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        got = {}
        for _ in procs:
            rank, msg, res = q.get(timeout=300)
            got[rank] = (msg, res)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(2):
        assert got[r][0] == "ok", f"rank {r}:\n{got[r][0]}"
        res = got[r][1]
        assert res["first_ok"] and res["first_status"] & 1 == 0 and res["first_async"] == 0, res
        assert res["timeout_ms"] == 1500, res
        assert res["ll_launches"] == (1 if count * 4 <= (64 << 10) else 0), res
    r0 = got[0][1]
    assert r0["lost_rc"] == 0  # stream-ordered: the call that enqueued the lost barrier had already returned
    assert r0["lost_status"] & 1 == 1
    # bits 8+: bit length of the call's longest wait in polls (~100 ns each): a 1.5 s wait is millions of polls
    assert (r0["lost_status"] >> 8) >= 16, hex(r0["lost_status"])
    assert 1.0 < r0["lost_s"] < 15.0, r0
    assert r0["async_after_lost"] == H.HcclResult.HCCL_E_TIMEOUT, r0
    assert r0["next_rc"] == H.HcclResult.HCCL_E_TIMEOUT, r0
    assert r0["then_rc"] == H.HcclResult.HCCL_E_SUSPENDING, r0
    assert r0["rs_rc"] == H.HcclResult.HCCL_E_SUSPENDING, r0
    assert r0["async_later"] == H.HcclResult.HCCL_E_TIMEOUT, r0
    assert r0["after_s"] < 1.0, r0  # the gate enqueues nothing


# Calls of the default-staging test: (collective, elements per rank's input, in place). The large staging tier's areas
# are HCCL_BUFFSIZE / 2 (100 MiB at the default 200 MB, the reference's 2 x HCCL_BUFFSIZE for the four) or, with
# HCCL_AMD_IPC_STAGING_MIB=1000, the largest allocation the set-up makes (2 x 1000 MiB + 2 x 23.5 MiB, below the 2 GiB
# that hipIpcOpenMemHandle never returned for in r03). At n = 2 and 100 MiB areas a two-shot owner's slot holds
# 12.5 Mi int32 per staging round, so the 300 and 600 MiB AllReduces cross several round boundaries, in place and out
# of place; the 640 MiB ReduceScatter input crosses the alternate areas' boundaries (at 1000 MiB areas: one boundary
# for the 600 MiB AllReduces, several of the 23.5 MiB alternate areas for the ReduceScatter).
DEFAULT_STAGING_CALLS = [
    (AR, 1025, False),
    (AR, (300 << 20) // 4 + 3, False),  # the r03 call that once returned a wrong result on rank 0
    (AR, (600 << 20) // 4 + 5, False),
    (AR, (600 << 20) // 4 + 5, True),
    (RS, 2 * ((320 << 20) // 4 + 7), False),
    (AR, 4097, True),
]


def _mismatch_detail(torch, y, want, xs_fn, prev, count, n, k, area_bytes):
    """Everything a wrong result can say about its cause: how many elements, where (owner chunk and
    staging round of the first, owners of all), the values at the first, and what the wrong value equals: the fold
    with one rank's operand missing, the previous call's result, zero, or none of these."""
    bad = (y != want).nonzero().flatten()
    i = int(bad[0])
    es, align = 4, 32  # int32; chunks rounded up to 128 B (HCCL_MIN_SLICE_ALIGN)
    chunk = ((count + n - 1) // n + align - 1) // align * align
    slot = area_bytes // es // n // 4 * 4  # elements of one owner's slot per staging round
    owners = torch.bincount(torch.div(bad, chunk, rounding_mode="floor"), minlength=n).tolist()
    got_i, want_i = int(y[i]), int(want[i])
    missing = [q for q in range(n) if got_i == want_i - int(xs_fn(q, i))]
    return {"call": k, "count": count, "bad": int(bad.numel()), "first": i, "last": int(bad[-1]),
            "first_owner": i // chunk, "first_round": (i % chunk) // slot, "bad_per_owner": owners,
            "got": got_i, "want": want_i, "missing_operand_of_rank": missing,
            "equals_previous_call": prev is not None and i < prev.numel() and got_i == int(prev[i]),
            "is_zero": got_i == 0}


def _default_staging_main(rank, n, port, q, area_mib):
    # area_mib None: the default large tier (HCCL_BUFFSIZE / 2 per area); 1000: one allocation of 2047 MiB per rank
    # (a 2 GiB one, r03's first layout, was never opened with hipIpcOpenMemHandle, so the rank-mode set-up hung)
    os.environ.pop("HCCL_AMD_IPC_STAGING_MIB", None)
    os.environ.pop("HCCL_BUFFSIZE", None)
    if area_mib is not None:
        os.environ["HCCL_AMD_IPC_STAGING_MIB"] = str(area_mib)
    os.environ["HCCL_AMD_IPC_TIMEOUT_MS"] = "20000"
    try:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=n,
                                timeout=datetime.timedelta(seconds=120))
        torch.cuda.set_device(0)
        import hccl_amd as H

        def all_gather(b):
            out = [None] * n
            dist.all_gather_object(out, b)
            return out

        comm = H.comm_init_host_exchange(n, rank, all_gather)
        comm.set_algo(H.Algo.IPC_TWOSHOT)
        s = torch.cuda.Stream()
        res = []
        prev = None
        for k, (kind, count, inplace) in enumerate(DEFAULT_STAGING_CALLS):
            # values distinct per call (1000 k), so a result left over from an earlier call is recognisable
            base = torch.arange(count, device="cuda", dtype=torch.int32) % 1000 + 1000 * k
            x = base + rank
            y = x if inplace else torch.full_like(x, -7)
            out_len = count // n if kind == RS else count
            if kind == RS:
                y = torch.full((out_len,), -7, dtype=torch.int32, device="cuda")
            torch.cuda.synchronize()  # x was made on the current stream; the collective runs on s
            if kind == RS:
                comm.reduce_scatter(x, y, H.HcclReduceOp.SUM, s)
                want = base[rank * out_len:(rank + 1) * out_len] * n + n * (n - 1) // 2
                xs_fn = (lambda qq, i, b0=base, o=rank * out_len: int(b0[o + i]) + qq)
            else:
                comm.all_reduce(x, y, H.HcclReduceOp.SUM, s)
                want = base * n + n * (n - 1) // 2
                xs_fn = (lambda qq, i, b0=base: int(b0[i]) + qq)
            s.synchronize()
            ok = bool(torch.equal(y, want))
            res.append((H.Algo(comm.last_algo).name, ok, comm.ipc_status() & 1))
            if not ok:
                res.append(("mismatch", _mismatch_detail(torch, y, want, xs_fn, prev, out_len, n, k,
                                                         (area_mib or 100) << 20)))
            prev = y.clone() if kind == AR else None
            del x, y, want, base
        dist.barrier()
        comm.destroy()
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception:  # noqa: BLE001
        q.put((rank, traceback.format_exc(), None))
        time.sleep(10)


@pytest.mark.timeout(240)
@pytest.mark.parametrize("area_mib", [None, 1000])
def test_ipc_rank_mode_default_staging(area_mib):
    """Rank mode with the default large staging tier (HCCL_BUFFSIZE / 2 per area) and with the largest one (1000 MiB
    areas: one allocation just below 2 GiB per rank, opened by every peer): two-shot AllReduces and a ReduceScatter
    exact without a barrier timeout, including calls that cross the areas' round boundaries in place and out of place.
    A wrong result reports everything it can say about its cause (_mismatch_detail) in the assertion message, in
    full."""
    n = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_default_staging_main, args=(r, n, port, q, area_mib)) for r in range(n)]
    for p in procs:
        p.start()
    try:
        got = {}
        for _ in procs:
            rank, msg, res = q.get(timeout=200)
            got[rank] = (msg, res)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    import json
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/ipc_default_staging_{area_mib or 'default'}.json", "w") as f:
        json.dump({str(r): got[r] for r in got}, f, indent=1)
    for r in range(n):
        assert got[r][0] == "ok", f"rank {r}:\n{got[r][0]}"
    # every rank's record in full, whichever rank is wrong (pytest would truncate a list diff)
    detail = json.dumps({r: got[r][1] for r in range(n)})
    for r in range(n):
        assert got[r][1] == [("IPC_TWOSHOT", True, 0)] * len(DEFAULT_STAGING_CALLS), detail


def _alternating_main(rank, n, port, q, calls, count):
    os.environ["HCCL_AMD_IPC_TIMEOUT_MS"] = "20000"
    try:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=n,
                                timeout=datetime.timedelta(seconds=120))
        torch.cuda.set_device(0)
        import hccl_amd as H

        def all_gather(b):
            out = [None] * n
            dist.all_gather_object(out, b)
            return out

        comm = H.comm_init_host_exchange(n, rank, all_gather)
        comm.set_algo(H.Algo.IPC)  # the auto family's order, the path the small-call rule takes
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        # integer-valued fp32: every order gives the same bits, so a wrong value can only be a call that ran into
        # another call's staging
        xs = [torch.full((count,), float((rank + 1) * (k + 1)), device="cuda") for k in range(calls)]
        ys = [torch.full((count,), -1.0, device="cuda") for _ in range(calls)]
        comm.all_reduce(xs[0], ys[0], H.HcclReduceOp.SUM, stream=streams[0])  # the collective set-up
        torch.cuda.synchronize()
        dist.barrier()
        for k in range(calls):  # back to back, alternating streams, no host wait
            comm.all_reduce(xs[k], ys[k], H.HcclReduceOp.SUM, stream=streams[k % 2])
        torch.cuda.synchronize()
        tot = n * (n + 1) // 2
        bad = [k for k in range(calls) if not bool(torch.all(ys[k] == float(tot * (k + 1))).item())]
        res = {"bad_calls": bad, "algo": H.Algo(comm.last_algo).name, "status_bit0": comm.ipc_status() & 1}
        dist.barrier()
        comm.destroy()
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception:  # noqa: BLE001
        q.put((rank, traceback.format_exc(), None))
        time.sleep(10)


@pytest.mark.timeout(240)
@pytest.mark.parametrize("count", [256, (1 << 20) // 4, (8 << 20) // 4 + 3])
def test_rank_mode_calls_on_alternating_streams_are_ordered(count):
    """Rank mode, the one-sided kernel: 32 AllReduces of one communicator issued back to back on two streams in turn
    with no host wait. Every call shares the communicator's staging, so each waits for the previous call's end through
    the communicator's tail event (EntryScope, recorded without the system-scope fence since r05): every
    result exact, no barrier timeout. 1 KiB and 1 MiB are the small-call rule's range, 8 MiB a two-shot call."""
    n, calls = 2, 32
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_alternating_main, args=(r, n, port, q, calls, count)) for r in range(n)]
    for p in procs:
        p.start()
    try:
        got = {}
        for _ in procs:
            rank, msg, res = q.get(timeout=200)
            got[rank] = (msg, res)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(n):
        assert got[r][0] == "ok", f"rank {r}:\n{got[r][0]}"
        assert got[r][1] == {"bad_calls": [], "algo": "IPC", "status_bit0": 0}, (r, got[r][1])
