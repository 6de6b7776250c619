"""The IPC plumbing the one-sided AllReduce relies on, across two processes on the one GPU: uncached device memory
(hipExtMallocWithFlags(hipDeviceMallocUncached)) exported with hipIpcGetMemHandle, opened in another process with
hipIpcOpenMemHandle(hipIpcMemLazyEnablePeerAccess), written there, read back by the owner. (On the 8-GPU node the
same calls run between devices; the flag protocol itself is covered by the loopback world in
test_gpu_collectives.py::test_ipc_allreduce_o2_and_status.)"""
import ctypes
import multiprocessing as mp
import os
import time

import pytest

pytestmark = pytest.mark.gpu


class IpcHandle(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_char * 64)]  # hipIpcMemHandle_t, passed BY VALUE to hipIpcOpenMemHandle


def _hip():
    import torch  # noqa: F401  (loads the HIP runtime torch uses)
    lib = ctypes.CDLL("libamdhip64.so.7", mode=ctypes.RTLD_GLOBAL)
    lib.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    lib.hipIpcGetMemHandle.argtypes = [ctypes.POINTER(IpcHandle), ctypes.c_void_p]
    lib.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), IpcHandle, ctypes.c_uint]
    lib.hipIpcCloseMemHandle.argtypes = [ctypes.c_void_p]
    lib.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    lib.hipSetDevice.argtypes = [ctypes.c_int]
    return lib


HIP_DEVICE_MALLOC_UNCACHED = 0x3
H2D, D2H = 1, 2
N = 1 << 20


def _owner(path, q):
    try:
        hip = _hip()
        assert hip.hipSetDevice(0) == 0
        p = ctypes.c_void_p()
        assert hip.hipExtMallocWithFlags(ctypes.byref(p), N * 4, HIP_DEVICE_MALLOC_UNCACHED) == 0
        zeros = (ctypes.c_uint32 * N)()
        assert hip.hipMemcpy(p, zeros, N * 4, H2D) == 0
        h = IpcHandle()
        assert hip.hipIpcGetMemHandle(ctypes.byref(h), p) == 0
        with open(path + ".tmp", "wb") as f:
            f.write(bytes(h))
        os.rename(path + ".tmp", path)
        t0 = time.time()
        while not os.path.exists(path + ".done"):
            assert time.time() - t0 < 120, "importer did not finish"
            time.sleep(0.05)
        back = (ctypes.c_uint32 * N)()
        assert hip.hipMemcpy(back, p, N * 4, D2H) == 0
        ok = all(back[i] == (i * 2654435761) & 0xFFFFFFFF for i in range(0, N, 997))
        q.put(("owner", "ok" if ok else "data mismatch"))
    except Exception as e:  # noqa: BLE001
        q.put(("owner", f"{type(e).__name__}: {e}"))


def _importer(path, q):
    try:
        hip = _hip()
        assert hip.hipSetDevice(0) == 0
        t0 = time.time()
        while not os.path.exists(path):
            assert time.time() - t0 < 120, "no handle"
            time.sleep(0.05)
        h = IpcHandle.from_buffer_copy(open(path, "rb").read())
        p = ctypes.c_void_p()
        rc = hip.hipIpcOpenMemHandle(ctypes.byref(p), h, 1)  # hipIpcMemLazyEnablePeerAccess
        assert rc == 0, f"hipIpcOpenMemHandle returned {rc}"
        data = (ctypes.c_uint32 * N)(*[(i * 2654435761) & 0xFFFFFFFF for i in range(N)])
        assert hip.hipMemcpy(p, data, N * 4, H2D) == 0
        assert hip.hipIpcCloseMemHandle(p) == 0
        open(path + ".done", "w").close()
        q.put(("importer", "ok"))
    except Exception as e:  # noqa: BLE001
        open(path + ".done", "w").close()
        q.put(("importer", f"{type(e).__name__}: {e}"))


def test_uncached_ipc_handle_roundtrip(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    path = str(tmp_path / "handle.bin")
    procs = [ctx.Process(target=_owner, args=(path, q)), ctx.Process(target=_importer, args=(path, q))]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {"owner": "ok", "importer": "ok"}, res
