"""torch.distributed backend "hccl" over libhccl_amd.so — the position of torch_npu's ProcessGroupHCCL.

The reference's Python caller (examples/03_ai_framework/01_pytorch/hccl_pytorch_allreduce_test.py:19-38) selects
the backend by name, ``dist.init_process_group(backend="hccl", ...)``, and reduces with ``dist.all_reduce``. Importing
this module registers that name, so the sample runs with only its device calls changed (``torch_npu.npu.set_device``
-> ``torch.cuda.set_device``, ``device="npu"`` -> ``"cuda"``)::

    import hccl_amd.process_group  # registers backend "hccl"
    dist.init_process_group(backend="hccl", rank=rank, world_size=world_size, init_method=init_method)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)

Every collective is one call of the C ABI (include/hccl.h) on a HIP stream; nothing here computes.
The mapping is the one ProcessGroupHCCL makes:

* ``all_reduce`` -> HcclAllReduce (in place, as torch requires; the reference allows sendBuf == recvBuf,
  all_reduce_auto_selector.cc:517-550);
* ``reduce`` -> HcclReduce (root = the group rank ``dst``);
* ``reduce_scatter_tensor`` / ``reduce_scatter`` -> HcclReduceScatter (input = rankSize blocks of the output's size,
  reduce_scatter_op.cc:158-159; the list form is packed into one buffer first), or HcclReduceScatterV when the list's
  blocks differ in size;
* ``all_gather_into_tensor`` / ``all_gather`` -> HcclAllGather;
* ``barrier`` -> a one-element HcclAllReduce, then the host waits for it;
* ``broadcast`` -> HcclAllGather of the tensor's bytes, keeping the root's block (for DDP's start-up sync; the reduce
  path has no broadcast of its own).

Reduce ops are HCCL's four (SUM, PRODUCT, MAX, MIN; hccl_types.h HcclReduceOp); AVG, PREMUL_SUM and the bitwise ops
have no HCCL counterpart and raise ValueError, as does any dtype HCCL does not reduce (the entry answers
HCCL_E_NOT_SUPPORT, which surfaces as HcclError).

The communicator is created on first use, on the device of the first tensor (as ProcessGroupHCCL does): rank 0 calls
HcclGetRootInfo and publishes the blob through the process group's store, every rank then calls
HcclCommInitRootInfo (examples/02_collectives/01_allreduce/main.cc:122-136 with the store as the out-of-band channel).
``HCCL_AMD_PG_TRANSPORT=ipc`` instead makes the IPC-only communicator (HcclAmdCommInitHostExchange) bootstrapped
through the store; several ranks may then share one GPU (RCCL refuses that), which is how tests/ run the multi-rank
form on a one-GPU box.

Streams are the NCCL backend's: each group owns one stream per device (the HCCL entries reject the null stream,
as the reference's do, and torch's default stream is the null stream). A collective waits there for the caller's
current stream, runs, and marks its tensors as used on that stream for the caching allocator; ``wait()`` makes the
then-current stream wait for it. The host never blocks except in ``barrier``. Under HIP-graph capture the call goes
on the capturing stream itself.
"""
from __future__ import annotations

import datetime
import os
import threading
import time
from typing import Callable, List, Optional

import torch
import torch.distributed as dist

import hccl_amd as H

BACKEND_NAME = "hccl"

_OPS = {
    dist.ReduceOp.SUM: H.HcclReduceOp.SUM,
    dist.ReduceOp.PRODUCT: H.HcclReduceOp.PROD,
    dist.ReduceOp.MAX: H.HcclReduceOp.MAX,
    dist.ReduceOp.MIN: H.HcclReduceOp.MIN,
}


def hccl_op(reduce_op) -> int:
    """HcclReduceOp for a torch ReduceOp (SUM/PRODUCT/MAX/MIN); ValueError for the ones HCCL lacks."""
    for k, v in _OPS.items():
        if reduce_op == k:
            return int(v)
    raise ValueError(f"backend {BACKEND_NAME!r} supports ReduceOp SUM, PRODUCT, MAX and MIN (HcclReduceOp); "
                     f"got {reduce_op}")


def output_dtype_mismatch(outputs: List[torch.Tensor], inp: torch.Tensor) -> bool:
    return any(o.numel() != inp.numel() or o.dtype != inp.dtype or o.device != inp.device for o in outputs)


class StoreAllGather:
    """Host all-gather of byte strings through a c10d Store: the bootstrap channel of the IPC-only communicator
    (HcclAmdHostAllGatherFn). Rounds are numbered, so every rank must call it the same number of times, which the
    library guarantees (it calls it only inside collective set-up)."""

    def __init__(self, store, rank: int, size: int, prefix: str):
        self.store, self.rank, self.size, self.prefix = store, rank, size, prefix
        self.round = 0

    def __call__(self, mine: bytes) -> List[bytes]:
        k = f"{self.prefix}/ag{self.round}"
        self.round += 1
        self.store.set(f"{k}/{self.rank}", mine)
        return [self.store.get(f"{k}/{r}") for r in range(self.size)]


class _Work(dist._Work):
    """Completion of one enqueued collective: an event recorded on the stream it was enqueued on, and a CUDA-aware
    future completed on that stream (its consumers' streams wait for it, as with the NCCL backend's futures; DDP's
    gradient hooks chain on it).

    Failures surface here as well as at the next collective: ``wait`` and ``is_success`` poll the communicator's
    asynchronous error (HcclGetCommAsyncError: an IPC barrier timeout, an RCCL-path execution timeout or an RCCL
    asynchronous error), and ``wait(timeout)`` blocks the host until the collective completes or the timeout passes,
    as ProcessGroupNCCL's work does."""

    def __init__(self, result: List[torch.Tensor], event: Optional[torch.cuda.Event],
                 future: Optional[torch.futures.Future] = None, comm: Optional["H.Comm"] = None):
        super().__init__()
        self._result = result
        self._event = event
        self._comm = comm
        if future is None:
            future = torch.futures.Future()
            future.set_result(result)
        self._future = future

    def _raise_async_error(self) -> None:
        if self._comm is not None and self._comm.handle:
            code = self._comm.async_error()
            if code != 0:
                raise H.HcclError("HcclGetCommAsyncError", code)

    def wait(self, timeout: Optional[datetime.timedelta] = None) -> bool:
        self._raise_async_error()
        if self._event is None:
            return True
        if timeout is not None and timeout.total_seconds() > 0:
            deadline = time.monotonic() + timeout.total_seconds()
            while not self._event.query():
                self._raise_async_error()
                if time.monotonic() > deadline:
                    raise RuntimeError(f"backend {BACKEND_NAME!r}: collective did not complete within {timeout}")
                time.sleep(0.001)
        torch.cuda.current_stream().wait_event(self._event)
        return True

    def is_completed(self) -> bool:
        return self._event is None or self._event.query()

    def is_success(self) -> bool:
        return self._comm is None or not self._comm.handle or self._comm.async_error() == 0

    def result(self) -> List[torch.Tensor]:
        return self._result

    def get_future(self) -> torch.futures.Future:
        return self._future


class ProcessGroupHCCL(dist.ProcessGroup):
    """One communicator per process group, created lazily on the first collective's device.

    Its bootstrap keys live under `prefix` in the store it is given. torch hands every group's backend a store of its
    own (a PrefixStore on the group's name, the same on every member), so the keys need no per-process numbering: a
    counter would differ between ranks once they take part in different subgroups (torch builds no backend on a rank
    outside a subgroup)."""

    def __init__(self, store, rank: int, size: int, timeout: datetime.timedelta,
                 comm_factory: Optional[Callable[[int], "H.Comm"]] = None, prefix: str = "hccl_amd"):
        super().__init__(rank, size)
        self._store = store
        self._timeout = timeout
        self._comm = None
        self._device: Optional[int] = None
        self._stream: Optional[torch.cuda.Stream] = None
        self._lock = threading.Lock()
        self._factory = comm_factory or self._make_comm
        self._prefix = prefix

    # ------------------------------------------------------------------------------------------------ communicator
    def _make_comm(self, device: int) -> "H.Comm":
        n, r = self.size(), self.rank()
        if os.environ.get("HCCL_AMD_PG_TRANSPORT", "").lower() == "ipc":
            c = H.comm_init_host_exchange(n, r, StoreAllGather(self._store, r, n, self._prefix))
            c.set_algo(H.Algo.IPC)  # the reference's default selection, so the bits are those of the RCCL path
            return c
        key = f"{self._prefix}/root_info"
        if r == 0:
            self._store.set(key, H.get_root_info())
        blob = self._store.get(key)
        return H.comm_init_root_info(n, bytes(blob), r)

    def comm(self, device: Optional[torch.device] = None) -> "H.Comm":
        """The group's communicator (created on `device`, default the current device, on first use)."""
        with self._lock:
            if self._comm is None:
                idx = torch.cuda.current_device() if device is None or device.index is None else device.index
                with torch.cuda.device(idx):
                    self._comm = self._factory(idx)
                self._device = idx
            elif device is not None and device.index is not None and device.index != self._device:
                raise ValueError(f"backend {BACKEND_NAME!r}: this process group's communicator is on cuda:"
                                 f"{self._device}, got a tensor on {device}")
            return self._comm

    # ------------------------------------------------------------------------------------------------ helpers
    @staticmethod
    def _check(t: torch.Tensor, what: str) -> None:
        if not t.is_cuda:
            raise ValueError(f"backend {BACKEND_NAME!r}: {what} must be a GPU tensor, got {t.device}")
        if not t.is_contiguous():
            raise ValueError(f"backend {BACKEND_NAME!r}: {what} must be contiguous")

    def _run(self, result: List[torch.Tensor], device: torch.device, fn, used: List[torch.Tensor]) -> _Work:
        comm = self.comm(device)
        with torch.cuda.device(device):
            if torch.cuda.is_current_stream_capturing():
                # HIP-graph capture: the call goes on the capturing stream itself. Transport groups captured on a
                # stream forked from the capture crash graph instantiation on this ROCm, and the graph
                # orders everything after it anyway.
                cur = torch.cuda.current_stream()
                fn(comm, cur)
                fut = torch.futures.Future(devices=[torch.device("cuda", torch.cuda.current_device())])
                fut.set_result(result)
                return _Work(result, None, fut, comm)
            if self._stream is None:
                self._stream = torch.cuda.Stream()
            side = self._stream
            side.wait_stream(torch.cuda.current_stream())
            fn(comm, side)
            for t in used:
                t.record_stream(side)
            ev = torch.cuda.Event()
            ev.record(side)
            fut = torch.futures.Future(devices=[torch.device("cuda", torch.cuda.current_device())])
            with torch.cuda.stream(side):
                fut.set_result(result)  # marks the result ready on the group's stream
        return _Work(result, ev, fut, comm)

    # ------------------------------------------------------------------------------------------------ collectives
    def allreduce(self, tensors: List[torch.Tensor], opts) -> _Work:
        op = hccl_op(opts.reduceOp)
        for t in tensors:
            self._check(t, "all_reduce tensor")
        return self._run(tensors, tensors[0].device,
                         lambda c, s: [c.all_reduce(t, t, op, s) for t in tensors], tensors)

    def reduce(self, tensors: List[torch.Tensor], opts) -> _Work:
        op = hccl_op(opts.reduceOp)
        t = tensors[opts.rootTensor]
        self._check(t, "reduce tensor")
        return self._run(tensors, t.device, lambda c, s: c.reduce(t, t, opts.rootRank, op, s), [t])

    def _reduce_scatter_base(self, output: torch.Tensor, input: torch.Tensor, opts) -> _Work:
        op = hccl_op(opts.reduceOp)
        self._check(output, "reduce_scatter output")
        self._check(input, "reduce_scatter input")
        if input.numel() != output.numel() * self.size() or input.dtype != output.dtype:
            raise ValueError(f"backend {BACKEND_NAME!r}: reduce_scatter input must hold world_size x output "
                             f"elements of the output's dtype")
        return self._run([output], output.device, lambda c, s: c.reduce_scatter(input, output, op, s),
                         [input, output])

    def reduce_scatter(self, outputs: List[torch.Tensor], inputs: List[List[torch.Tensor]], opts) -> _Work:
        if len(outputs) != 1 or len(inputs) != 1 or len(inputs[0]) != self.size():
            raise ValueError(f"backend {BACKEND_NAME!r}: reduce_scatter takes one output and world_size inputs")
        parts, output = inputs[0], outputs[0]
        packed = torch.cat([x.reshape(-1) for x in parts])
        counts = [x.numel() for x in parts]
        if all(c == output.numel() for c in counts):
            return self._reduce_scatter_base(output, packed, opts)
        # uneven blocks: HcclReduceScatterV over the packed input (rank q's block at the running offset)
        op = hccl_op(opts.reduceOp)
        self._check(output, "reduce_scatter output")
        if output.numel() != counts[self.rank()] or any(x.dtype != output.dtype for x in parts):
            raise ValueError(f"backend {BACKEND_NAME!r}: reduce_scatter output must hold this rank's block")
        displs = [sum(counts[:q]) for q in range(len(counts))]
        return self._run([output], output.device,
                         lambda c, s: c.reduce_scatter_v(packed, counts, displs, output, op, s), [packed, output])

    def _allgather_base(self, output: torch.Tensor, input: torch.Tensor, opts) -> _Work:
        self._check(output, "all_gather output")
        self._check(input, "all_gather input")
        if output.numel() != input.numel() * self.size() or input.dtype != output.dtype:
            raise ValueError(f"backend {BACKEND_NAME!r}: all_gather output must hold world_size x input elements")
        return self._run([output], output.device, lambda c, s: c.all_gather(input, output, s),
                         [input, output])

    def allgather(self, outputs: List[List[torch.Tensor]], inputs: List[torch.Tensor], opts) -> _Work:
        if len(outputs) != 1 or len(inputs) != 1 or len(outputs[0]) != self.size():
            raise ValueError(f"backend {BACKEND_NAME!r}: all_gather takes one input and world_size outputs")
        inp = inputs[0]
        self._check(inp, "all_gather input")
        if output_dtype_mismatch(outputs[0], inp):
            raise ValueError(f"backend {BACKEND_NAME!r}: all_gather outputs must match the input's size and dtype")
        m = inp.numel()
        flat = torch.empty(m * self.size(), dtype=inp.dtype, device=inp.device)

        def gather_and_unpack(c, s):
            c.all_gather(inp, flat, s)
            with torch.cuda.stream(s):  # unpacked on the group's stream, after the gather
                for r, o in enumerate(outputs[0]):
                    o.copy_(flat[r * m:(r + 1) * m].view_as(o))

        return self._run(outputs[0], inp.device, gather_and_unpack, [inp, flat] + list(outputs[0]))

    def broadcast(self, tensors: List[torch.Tensor], opts) -> _Work:
        """Broadcast from opts.rootRank, built on HcclAllGather of the tensor's bytes (the reduce path has no
        broadcast of its own; DDP needs one at construction to sync module states): every rank gathers every rank's
        bytes and keeps the root's block, so the root's bits arrive unchanged whatever the dtype."""
        t = tensors[opts.rootTensor]
        self._check(t, "broadcast tensor")
        root = opts.rootRank
        raw = t.reshape(-1).view(torch.uint8)  # contiguous: a view (a 0-dim tensor has no byte view of its own)
        m = raw.numel()
        flat = torch.empty(m * self.size(), dtype=torch.uint8, device=t.device)

        def gather_root(c, s):
            c.all_gather(raw.reshape(-1), flat, s)
            with torch.cuda.stream(s):
                raw.reshape(-1).copy_(flat[root * m:(root + 1) * m])

        return self._run(tensors, t.device, gather_root, [t, flat])

    def barrier(self, opts) -> _Work:
        dev = torch.device("cuda", self._device if self._device is not None else torch.cuda.current_device())
        one = torch.ones(1, dtype=torch.int32, device=dev)
        work = self._run([one], dev, lambda c, s: c.all_reduce(one, one, H.HcclReduceOp.SUM, s),
                         [one])
        if work._event is not None:  # under capture there is nothing to wait for on the host
            work._event.synchronize()  # a barrier returns to the host only when every rank has arrived
        return work

    def getBackendName(self) -> str:
        return BACKEND_NAME

    def shutdown(self) -> None:
        """Called by dist.destroy_process_group: HcclCommDestroy (collective for IPC communicators)."""
        with self._lock:
            if self._comm is not None:
                if self._device is not None:
                    torch.cuda.synchronize(self._device)
                self._comm.destroy()
                self._comm = None


def _create(store, rank: int, size: int, timeout: datetime.timedelta) -> ProcessGroupHCCL:
    return ProcessGroupHCCL(store, rank, size, timeout)


def register(name: str = BACKEND_NAME) -> None:
    """Registers the backend under `name` for GPU tensors (registering again replaces the creator)."""
    dist.Backend.register_backend(name, _create, devices=["cuda"])


register()
