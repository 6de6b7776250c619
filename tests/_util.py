"""Shared helpers for the parity tests: numpy (oracle storage) <-> torch (device) conversion."""
import numpy as np
import torch

from oracle import oracle as O

_TORCH_OF = {
    O.INT8: torch.int8, O.INT16: torch.int16, O.INT32: torch.int32, O.INT64: torch.int64, O.UINT64: torch.uint64,
    O.FP16: torch.float16, O.BFP16: torch.bfloat16, O.FP32: torch.float32, O.FP64: torch.float64,
}


def torch_dtype(dtype: int):
    return _TORCH_OF[dtype]


def to_device(dtype: int, a: np.ndarray, device="cuda") -> torch.Tensor:
    a = np.ascontiguousarray(a)
    if dtype == O.FP16:
        t = torch.from_numpy(a.view(np.float16).copy())
    elif dtype == O.BFP16:
        t = torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16)
    else:
        t = torch.from_numpy(a.copy())
    return t.to(device)


def to_host(dtype: int, t: torch.Tensor) -> np.ndarray:
    t = t.detach().cpu().contiguous()
    if dtype == O.FP16:
        return t.view(torch.int16).numpy().view(np.uint16).copy()
    if dtype == O.BFP16:
        return t.view(torch.int16).numpy().view(np.uint16).copy()
    return t.numpy().copy()
