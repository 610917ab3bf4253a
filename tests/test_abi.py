"""The C-ABI library loads and exports every entry point include/migym.h declares
(no compute calls: runs without a GPU).  Also checks the ctypes/NumPy struct
mirrors match the C layouts."""
import os
import re

import pytest

from migym import _abi, model as M

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "migym.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mg_[a-z_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_abi.LIB_PATH):
        import subprocess
        import sys
        subprocess.check_call([sys.executable, os.path.join(ROOT, "__graft_entry__.py"), "build"])
    return _abi.lib()


def test_every_declared_symbol_is_exported(lib):
    syms = declared_symbols()
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_abi.EXPORTS), set(syms) ^ set(_abi.EXPORTS)


def test_struct_layouts_match(lib):
    _abi.check_layout(lib)
    assert lib.mg_model_sizeof() == M.MODEL_DTYPE.itemsize
    assert lib.mg_version() == 7


def test_bad_arguments_fail_loudly_without_device(lib):
    import ctypes as C
    h = C.c_void_p()
    rc = lib.mg_sim_create(None, None, 0, 0, C.byref(h))
    assert rc == -1
    assert b"bad arguments" in lib.mg_last_error()


def test_model_tables_roundtrip():
    for name in ("ant", "humanoid", "cartpole"):
        spec = M.load_builtin(name)
        packed = M.pack_model(spec)
        assert packed["num_nodes"] == len(spec.nodes)
        assert all(packed["parent"][i] < i for i in range(1, len(spec.nodes)))
