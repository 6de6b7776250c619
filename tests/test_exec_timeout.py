"""HCCL_EXEC_TIMEOUT -> the one-sided kernel's barrier bound (host logic only, no GPU).

The IPC kernel is the reference's AIV engine, so the variable follows the AIV-mode rule of
docs/zh/user_guide/hccl_env/HCCL_EXEC_TIMEOUT.md (seconds, 10-ms precision, default 1091, 0 or above 1091 -> 1091),
parsed with ParseExecTimeout's format check (src/common/alg_env_config.cc:43-110: digits, at most two decimals,
at most UINT32_MAX; malformed -> default). HCCL_AMD_IPC_TIMEOUT_MS, the tests' short bound, takes precedence."""
import pytest

import hccl_amd as H

DEFAULT_MS = 1091000


@pytest.mark.parametrize("value,ms", [
    (None, DEFAULT_MS), ("", DEFAULT_MS), ("0", DEFAULT_MS), ("1091", DEFAULT_MS), ("1092", DEFAULT_MS),
    ("4294967295", DEFAULT_MS), ("1", 1000), ("1.5", 1500), ("0.05", 50), ("600", 600000), ("12.25", 12250),
    # malformed: rejected by the reference's format check, so the default applies
    ("1.234", DEFAULT_MS), (".5", DEFAULT_MS), ("5.", DEFAULT_MS), ("-1", DEFAULT_MS), ("1e3", DEFAULT_MS),
    ("abc", DEFAULT_MS), ("4294967296", DEFAULT_MS), (" 5", DEFAULT_MS),
])
def test_exec_timeout_aiv_rule(monkeypatch, value, ms):
    monkeypatch.delenv("HCCL_AMD_IPC_TIMEOUT_MS", raising=False)
    if value is None:
        monkeypatch.delenv("HCCL_EXEC_TIMEOUT", raising=False)
    else:
        monkeypatch.setenv("HCCL_EXEC_TIMEOUT", value)
    assert H.lib.HcclAmdIpcTimeoutMs() == ms


def test_test_bound_takes_precedence(monkeypatch):
    monkeypatch.setenv("HCCL_EXEC_TIMEOUT", "30")
    monkeypatch.setenv("HCCL_AMD_IPC_TIMEOUT_MS", "1500")
    assert H.lib.HcclAmdIpcTimeoutMs() == 1500
    monkeypatch.setenv("HCCL_AMD_IPC_TIMEOUT_MS", "0")  # out of range: ignored
    assert H.lib.HcclAmdIpcTimeoutMs() == 30000


def test_async_error_rejects_null():
    assert H.lib.HcclGetCommAsyncError(None, None) == H.HcclResult.HCCL_E_PTR
