"""The RCCL p2p channel settings the library makes when it is loaded and asked to (HCCL_AMD_P2P_CHANNELS_PER_PEER; comm.cc
ConfigureRcclP2pChannels; opt-in since r05), host side only: each case loads the library in a fresh interpreter with a given environment and reads back what
HcclAmdRcclP2pChannels reports and what the C environment then holds (RCCL reads it at its first communicator).
The GPU side (RCCL honours them) is tests/test_gpu_rccl.py::test_rccl_p2p_channels_configured."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROBE = r"""
import ctypes, json
import hccl_amd as H
getenv = ctypes.CDLL(None).getenv
getenv.restype = ctypes.c_char_p
getenv.argtypes = [ctypes.c_char_p]
env = {k: (getenv(k.encode()) or b"").decode() or None for k in ("NCCL_NCHANNELS_PER_PEER", "NCCL_MIN_P2P_NCHANNELS")}
print(json.dumps({"reported": list(H.rccl_p2p_channels()), "env": env}))
"""


def probe(extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("NCCL_NCHANNELS_PER_PEER", "NCCL_MIN_P2P_NCHANNELS", "HCCL_AMD_P2P_CHANNELS_PER_PEER")}
    env.update(extra)
    out = subprocess.run([sys.executable, "-c", PROBE], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    return json.loads(out.stdout.strip().splitlines()[-1])


OPT16 = {"HCCL_AMD_P2P_CHANNELS_PER_PEER": "16"}


@pytest.mark.parametrize("extra,reported,env", [
    ({}, [0, 0], {"NCCL_NCHANNELS_PER_PEER": None, "NCCL_MIN_P2P_NCHANNELS": None}),
    (OPT16, [16, 64], {"NCCL_NCHANNELS_PER_PEER": "16", "NCCL_MIN_P2P_NCHANNELS": "64"}),
    ({"HCCL_AMD_P2P_CHANNELS_PER_PEER": "4"}, [4, 32], {"NCCL_NCHANNELS_PER_PEER": "4", "NCCL_MIN_P2P_NCHANNELS": "32"}),
    ({"HCCL_AMD_P2P_CHANNELS_PER_PEER": "3"}, [4, 32], {"NCCL_NCHANNELS_PER_PEER": "4", "NCCL_MIN_P2P_NCHANNELS": "32"}),
    ({"HCCL_AMD_P2P_CHANNELS_PER_PEER": "1"}, [1, 8], {"NCCL_NCHANNELS_PER_PEER": "1", "NCCL_MIN_P2P_NCHANNELS": "8"}),
    ({"HCCL_AMD_P2P_CHANNELS_PER_PEER": "0"}, [0, 0], {"NCCL_NCHANNELS_PER_PEER": None, "NCCL_MIN_P2P_NCHANNELS": None}),
    ({"NCCL_NCHANNELS_PER_PEER": "2"}, [2, 0], {"NCCL_NCHANNELS_PER_PEER": "2", "NCCL_MIN_P2P_NCHANNELS": None}),
    # the per-peer value in effect is the caller's 2: minimum 2 x 7 rounded up, not 16 x 7
    (dict(OPT16, NCCL_NCHANNELS_PER_PEER="2"), [2, 16], {"NCCL_NCHANNELS_PER_PEER": "2", "NCCL_MIN_P2P_NCHANNELS": "16"}),
    (dict(OPT16, NCCL_NCHANNELS_PER_PEER="2", NCCL_MIN_P2P_NCHANNELS="8"), [2, 8],
     {"NCCL_NCHANNELS_PER_PEER": "2", "NCCL_MIN_P2P_NCHANNELS": "8"}),
], ids=["default_untouched", "opt_in_16", "four", "rounded_up", "one", "zero", "caller_per_peer_only",
        "caller_per_peer_with_opt_in", "caller_both"])
def test_p2p_channel_settings_at_load(extra, reported, env):
    got = probe(extra)
    assert got["reported"] == reported, got
    assert got["env"] == env, got
