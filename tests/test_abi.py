"""The C ABI (include/factmx.h) vs the built library and its ctypes binding (CPU-only).

No compute is launched: only symbol export, ABI version, argument counts, and the
host-side argument validation that runs before any HIP call.
"""
import ctypes
import os
import re
import subprocess

import pytest

from factmx import native as nx

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "factmx.h")


def _declarations():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    decls = {}
    for m in re.finditer(r"\b(?:int|void\s*\*|void|long long|const char\s*\*)\s*(fx_\w+)\s*\(([^;{]*?)\)\s*;", src, flags=re.S):
        args = m.group(2).strip()
        n = 0 if args in ("", "void") else len([a for a in args.split(",") if a.strip()])
        decls[m.group(1)] = n
    return decls


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(nx.LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(ROOT, "fact-clip_amd", "csrc"), "-j8"], check=True,
                       stdout=subprocess.DEVNULL)
    return nx.load()


def test_header_matches_binding():
    decls = _declarations()
    assert len(decls) >= 30
    assert set(decls) == set(nx.SIGNATURES), (set(decls) ^ set(nx.SIGNATURES))
    for name, n in decls.items():
        assert len(nx.SIGNATURES[name][1]) == n, (name, n, len(nx.SIGNATURES[name][1]))


def test_library_exports_every_symbol(lib):
    raw = ctypes.CDLL(nx.LIB_PATH)
    for name in _declarations():
        assert hasattr(raw, name), name
    assert lib.fx_version() == nx.ABI_VERSION


def test_struct_layouts():
    # fx_operand / fx_gemm_desc field lists mirror the header order (sizes are what the C side reads)
    src = open(HEADER).read()
    for struct, cls in (("fx_operand", nx.Operand), ("fx_gemm_desc", nx.GemmDesc),
                        ("fx_mstcn_params", nx.MstcnParams), ("fx_mstcn_grads", nx.MstcnGrads)):
        body = re.search(r"typedef struct\s+" + struct + r"\s*\{(.*?)\}\s*" + struct + r"\s*;", src, flags=re.S).group(1)
        body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
        body = re.sub(r"//[^\n]*", "", body)
        names = []
        for stmt in body.split(";"):
            names += re.findall(r"(\w+)\s*(?:,|$)", stmt.strip())
        assert names == [f[0] for f in cls._fields_], (struct, names)


def test_gemm_validation_without_gpu(lib):
    d = nx.GemmDesc()
    d.M, d.N, d.K, d.batch = 0, 8, 8, 1
    assert lib.fx_gemm(ctypes.byref(d), None) == 0          # empty problem: nothing to launch
    d.M = 8
    st = lib.fx_gemm(ctypes.byref(d), None)                 # null operands are rejected before any HIP call
    assert st < 0 and b"null operand" in lib.fx_last_error()
    d.batch = 0
    assert lib.fx_gemm(ctypes.byref(d), None) < 0 and b"bad sizes" in lib.fx_last_error()


def test_workspace_queries(lib):
    d = nx.GemmDesc()
    d.M, d.N, d.K, d.batch, d.split_k = 256, 769, 4096, 1, 7
    assert lib.fx_gemm_workspace_floats(ctypes.byref(d)) == 7 * 256 * 769
    d.split_k = 1
    assert lib.fx_gemm_workspace_floats(ctypes.byref(d)) == 0
    assert lib.fx_gru_saved_floats(121, 256) > 0


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(nx, "_lib", None)
    with pytest.raises(nx.FactmxNativeError):
        nx.load(str(tmp_path / "nope.so"))
