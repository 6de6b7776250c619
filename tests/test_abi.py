"""The drop-in boundary without a GPU: every symbol include/*.h declares is exported by libhccl_amd.so with the
ctypes signature the Python mirror uses; enum numbering is pinned to the reference's tables; the entry checks that
run before any device work return the reference's codes (all_reduce_op.cc:37,135-157; reduce_scatter_op.cc:47;
reduce_op.cc:106-127).
"""
import os
import re
import subprocess

import pytest

import hccl_amd as H

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("hccl.h", "hccl_amd.h")]


def declared():
    out = {}
    for h in HEADERS:
        text = open(h).read()
        for m in re.finditer(r"extern\s+[\w\s\*]+?\b(Hccl\w+)\s*\(([^;]*?)\)\s*;", text, re.S):
            args = [a for a in m.group(2).split(",") if a.strip() and a.strip() != "void"]
            out[m.group(1)] = len(args)
    return out


def test_every_declared_symbol_is_exported_with_matching_arity():
    decl = declared()
    assert len(decl) >= 19
    nm = subprocess.run(["nm", "-D", "--defined-only", H.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (Hccl\w+)", nm))
    for name, nargs in decl.items():
        assert name in exported, f"{name} declared but not exported"
        assert name in H.SIGNATURES, f"{name} missing from the ctypes table"
        assert len(H.SIGNATURES[name][1]) == nargs, name
        assert getattr(H.lib, name) is not None


def test_reference_operator_signatures_are_kept():
    """Same names, argument order and types as /root/reference/include/hccl.h:35-37, 67-69, 245-247."""
    text = open(HEADERS[0]).read()
    squash = " ".join(text.split())
    assert ("HcclResult HcclAllReduce(void* sendBuf, void* recvBuf, uint64_t count, HcclDataType dataType, "
            "HcclReduceOp op, HcclComm comm, aclrtStream stream);") in squash
    assert ("HcclResult HcclReduceScatter(void* sendBuf, void* recvBuf, uint64_t recvCount, HcclDataType dataType, "
            "HcclReduceOp op, HcclComm comm, aclrtStream stream);") in squash
    assert ("HcclResult HcclReduce(void* sendBuf, void* recvBuf, uint64_t count, HcclDataType dataType, "
            "HcclReduceOp op, uint32_t root, HcclComm comm, aclrtStream stream);") in squash


def _enum_values(header, prefix):
    text = open(os.path.join(ROOT, "include", header)).read()
    return {m.group(1): int(m.group(2)) for m in re.finditer(rf"\b({prefix}\w+)\s*=\s*(\d+)", text)}


def test_datatype_numbering_matches_reference_tables():
    """DATATYPE_SIZE_TABLE order (alg_param.h:43-61) and VALID_HCCL_DATA_TYPES (hccl_common.h:60-67)."""
    v = _enum_values("hccl_types.h", "HCCL_DATA_TYPE_")
    order = ["INT8", "INT16", "INT32", "FP16", "FP32", "INT64", "UINT64", "UINT8", "UINT16", "UINT32", "FP64",
             "BFP16", "INT128"]
    for i, name in enumerate(order):
        assert v["HCCL_DATA_TYPE_" + name] == i
        assert H.HcclDataType[name] == i
    assert v["HCCL_DATA_TYPE_HIF8"] == 14 and v["HCCL_DATA_TYPE_FP8E8M0"] == 17
    assert v["HCCL_DATA_TYPE_RESERVED"] == 255
    sizes = [1, 2, 4, 2, 4, 8, 8, 1, 2, 4, 8, 2, 16]
    for i, sz in enumerate(sizes):
        assert H.lib.HcclAmdDataTypeSize(i) == sz


def test_reduce_op_and_result_numbering():
    ops = _enum_values("hccl_types.h", "HCCL_REDUCE_")
    assert ops == {"HCCL_REDUCE_SUM": 0, "HCCL_REDUCE_PROD": 1, "HCCL_REDUCE_MAX": 2, "HCCL_REDUCE_MIN": 3,
                   "HCCL_REDUCE_RESERVED": 4}
    res = _enum_values("hccl_types.h", "HCCL_E_")
    for name, val in res.items():
        assert H.HcclResult[name] == val
    assert H.lib.HcclAmdGetErrorString(2) == b"HCCL_E_PTR"


def test_entry_checks_before_device_work():
    L, E = H.lib, H.HcclResult
    FP32 = H.HcclDataType.FP32
    p = 0x1000  # never dereferenced: every call below returns before touching memory
    assert L.HcclAllReduce(None, None, 0, FP32, 0, None, None) == E.HCCL_SUCCESS        # count 0 short-circuits
    assert L.HcclAllReduce(p, p, 8, FP32, 0, p, None) == E.HCCL_E_PTR                   # stream first
    assert L.HcclAllReduce(p, p, 8, FP32, 0, None, p) == E.HCCL_E_PTR                   # then comm
    assert L.HcclAllReduce(None, p, 8, FP32, 0, p, p) == E.HCCL_E_PTR                   # sendBuf
    assert L.HcclAllReduce(p, None, 8, FP32, 0, p, p) == E.HCCL_E_PTR                   # recvBuf
    assert L.HcclReduceScatter(None, None, 0, FP32, 0, None, None) == E.HCCL_SUCCESS
    assert L.HcclReduceScatter(p, p, 8, FP32, 0, None, p) == E.HCCL_E_PTR
    assert L.HcclReduce(None, None, 0, FP32, 0, 0, None, None) == E.HCCL_SUCCESS
    assert L.HcclReduce(p, p, 8, FP32, 0, 0, None, p) == E.HCCL_E_PTR                   # comm first for Reduce
    assert L.HcclCommDestroy(None) == E.HCCL_E_PTR
    assert L.HcclGetRootInfo(None) == E.HCCL_E_PTR


def test_build_schedule_rejects_bad_parameters():
    import ctypes
    n = ctypes.c_uint64(0)
    L, E = H.lib, H.HcclResult
    assert L.HcclAmdBuildSchedule(0, 0, 4, 4, 100, 4, 0, 0, None, 0, ctypes.byref(n), None, None) == E.HCCL_E_PARA
    assert L.HcclAmdBuildSchedule(2, 0, 4, 0, 100, 4, 9, 0, None, 0, ctypes.byref(n), None, None) == E.HCCL_E_PARA
    assert L.HcclAmdBuildSchedule(0, 0, 4, 0, 100, 13, 0, 0, None, 0, ctypes.byref(n), None, None) == \
        E.HCCL_E_NOT_SUPPORT
    assert L.HcclAmdBuildSchedule(0, 0, 4, 0, 100, 4, 0, 0, None, 0, None, None, None) == E.HCCL_E_PTR


def test_product_does_not_link_the_oracle():
    """libhccl_amd.so must not depend on, or contain, the CPU oracle (no CPU fallback path)."""
    out = subprocess.run(["readelf", "-d", H.LIB_PATH], capture_output=True, text=True, check=True).stdout
    assert "oracle" not in out
    nm = subprocess.run(["nm", "-D", H.LIB_PATH], capture_output=True, text=True, check=True).stdout
    assert "orc_" not in nm


@pytest.mark.parametrize("header", ["hccl.h", "hccl_types.h", "hccl_amd.h"])
def test_headers_compile_as_plain_c(header, tmp_path):
    src = tmp_path / "t.c"
    src.write_text(f'#include "{header}"\nint main(void) {{ return 0; }}\n')
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(src), "-o",
                    str(tmp_path / "t")], check=True)


def test_c_caller_links_and_gets_reference_codes(tmp_path):
    """A plain C caller, written the way the reference's samples call HCCL (examples/02_collectives/01_allreduce/
    main.cc), compiles against include/hccl.h, links libhccl_amd.so and gets the reference's entry-check codes
    (no device work: every call returns before touching memory)."""
    src = tmp_path / "caller.c"
    src.write_text(r'''
#include <stdio.h>
#include "hccl.h"
int main(void) {
    void* p = (void*)0x1000;
    int bad = 0;
    bad |= HcclAllReduce(NULL, NULL, 0, HCCL_DATA_TYPE_FP32, HCCL_REDUCE_SUM, NULL, NULL) != HCCL_SUCCESS;
    bad |= HcclAllReduce(p, p, 8, HCCL_DATA_TYPE_FP32, HCCL_REDUCE_SUM, p, NULL) != HCCL_E_PTR;
    bad |= HcclReduceScatter(p, p, 8, HCCL_DATA_TYPE_BFP16, HCCL_REDUCE_SUM, NULL, p) != HCCL_E_PTR;
    bad |= HcclReduce(p, p, 8, HCCL_DATA_TYPE_FP16, HCCL_REDUCE_MAX, 0, NULL, p) != HCCL_E_PTR;
    bad |= HcclAllGather(p, p, 8, HCCL_DATA_TYPE_INT8, NULL, p) != HCCL_E_PTR;
    bad |= HcclGetRootInfo(NULL) != HCCL_E_PTR;
    uint32_t n = 0;
    bad |= HcclGetRankSize(NULL, &n) != HCCL_E_PTR;
    printf("%s\n", bad ? "FAIL" : "OK");
    return bad;
}
''')
    exe = tmp_path / "caller"
    libdir = os.path.dirname(H.LIB_PATH)
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(src), "-o",
                    str(exe), "-L", libdir, "-lhccl_amd", f"-Wl,-rpath,{libdir}"], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.strip() == "OK", (out.stdout, out.stderr)


def test_missing_library_fails_loudly(tmp_path):
    """No fallback: with the shared object absent, importing the package raises instead of running anything else.
    Checked on a copy of the package in a scratch directory, so the real build is untouched."""
    import shutil
    pkg = tmp_path / "hccl_amd"
    shutil.copytree(os.path.join(ROOT, "hccl_amd"), pkg,
                    ignore=shutil.ignore_patterns("*.so", "build", "csrc", "__pycache__", "Makefile"))
    code = "import hccl_amd"
    out = subprocess.run([os.sys.executable, "-c", code], cwd=str(tmp_path), capture_output=True, text=True,
                         timeout=300)
    assert out.returncode != 0
    assert "ImportError" in out.stderr and "no fallback" in out.stderr, out.stderr[-2000:]
