"""HcclCommInitClusterInfo's rank table handling (hccl_amd/csrc/bootstrap.cc), on the CPU: the JSON cluster
description of the reference's docs (cluster_info_config/rank_table_config_a2.md / _a3.md: "status", "server_list",
per-device "device_id" / "rank_id" as strings, optional "host_ip" / "host_port"), parsed and validated through
HcclAmdRankTableInfo. The tables below are written for these tests in that format."""
import json

import pytest

import hccl_amd as H
from hccl_amd._lib import HcclError


def _table(servers, status="completed", version="1.0"):
    return {"status": status, "version": version, "server_count": str(len(servers)), "server_list": servers}


def _server(sid, devices, host_ip=None):
    s = {"server_id": sid, "device": devices}
    if host_ip is not None:
        s["host_ip"] = host_ip
    return s


def _dev(dev, rank, **extra):
    d = {"device_id": str(dev), "device_ip": f"192.168.1.{10 + rank}", "device_port": "16667", "rank_id": str(rank)}
    d.update(extra)
    return d


def _write(tmp_path, obj, name="ranktable.json"):
    p = tmp_path / name
    p.write_text(json.dumps(obj, indent=2) if not isinstance(obj, str) else obj)
    return str(p)


def test_two_servers_two_devices(tmp_path):
    t = _table([_server("node_0", [_dev(0, 0), _dev(1, 1)]), _server("node_1", [_dev(0, 2), _dev(1, 3)])])
    path = _write(tmp_path, t)
    assert [H.rank_table_info(path, r) for r in range(4)] == [(4, 0), (4, 1), (4, 0), (4, 1)]


def test_single_server_eight_devices_any_order(tmp_path):
    devs = [_dev(d, 7 - d) for d in range(8)]  # rank_id need not follow list order
    path = _write(tmp_path, _table([_server("node_0", devs)]))
    for r in range(8):
        assert H.rank_table_info(path, r) == (8, 7 - r)


def test_super_pod_fields_and_numeric_values(tmp_path):
    """A3-style entries (host_ip per server, host_port / super_device_id per device) and numbers instead of strings."""
    devs = [{"device_id": d, "super_device_id": str(d), "host_port": 16665 + d, "rank_id": d} for d in range(4)]
    path = _write(tmp_path, _table([_server("node_0", devs, host_ip="127.0.0.1")], version="1.2"))
    assert H.rank_table_info(path, 3) == (4, 3)


@pytest.mark.parametrize("mutate,why", [
    (lambda t: t.update(status="initializing"), "status not completed"),
    (lambda t: t["server_list"][0]["device"][1].update(rank_id="0"), "repeated rank_id"),
    (lambda t: t["server_list"][0]["device"][1].update(rank_id="5"), "rank_id out of range"),
    (lambda t: t["server_list"][0]["device"][0].pop("device_id"), "missing device_id"),
    (lambda t: t["server_list"][0]["device"][0].update(rank_id="-1"), "negative rank_id"),
    (lambda t: t.update(server_list=[]), "empty server_list"),
    (lambda t: t["server_list"][0].pop("device"), "server without devices"),
])
def test_invalid_tables_are_rejected(tmp_path, mutate, why):
    t = _table([_server("node_0", [_dev(0, 0), _dev(1, 1)])])
    mutate(t)
    path = _write(tmp_path, t)
    with pytest.raises(HcclError, match="HCCL_E_PARA"):
        H.rank_table_info(path, 0)


@pytest.mark.parametrize("text", ['{"status": "completed", "server_list": [', "not json", "",
                                  '{"status": "completed", "server_list": [{"device": [{"rank_id": "0", '
                                  '"device_id": "0"}]}]} trailing'])
def test_malformed_json_is_rejected(tmp_path, text):
    path = _write(tmp_path, text)
    with pytest.raises(HcclError, match="HCCL_E_PARA"):
        H.rank_table_info(path, 0)


def test_rank_outside_table_and_missing_file(tmp_path):
    path = _write(tmp_path, _table([_server("node_0", [_dev(0, 0), _dev(1, 1)])]))
    with pytest.raises(HcclError, match="HCCL_E_PARA"):
        H.rank_table_info(path, 2)
    with pytest.raises(HcclError, match="HCCL_E_PARA"):
        H.rank_table_info(str(tmp_path / "absent.json"), 0)


def test_json_escapes_and_whitespace(tmp_path):
    text = ('\n {"status" :"completed","version":"1.0","server_list":[ {"server_id":"n\\u006fde\\t0","device":'
            '[{"device_id":"0","rank_id":"0","note":"a\\"b\\\\c"}]}]}\n')
    path = _write(tmp_path, text)
    assert H.rank_table_info(path, 0) == (1, 0)
