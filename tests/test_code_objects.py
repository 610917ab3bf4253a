"""The shipped libmigym.so's device code has no real calls (CPU test: disassembles the gfx950 code objects).

Every team-kernel phase is force-inlined: round 3 saw a real call into the narrowphase
miscompile with this toolchain, and the inliner has declined a forceinline before.  A declined inline would
bring that bug class back silently, so this test (and build.py, at link time) disassembles every code object
of the library and asserts that no ``s_swappc_b64`` call and no callable function (``s_setpc_b64 s[30:31]``
return) is left.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "isaacgymenvs-ma_amd")
sys.path.insert(0, PKG)
import codeobj  # noqa: E402

SO = os.path.join(PKG, "migym", "_lib", "libmigym.so")


@pytest.mark.skipif(not codeobj.have_objdump(), reason="llvm-objdump not installed")
def test_shipped_library_has_no_device_calls():
    assert os.path.exists(SO), "build first (__graft_entry__.build)"
    cos = codeobj.device_code_objects(SO)
    assert len(cos) >= 2, "expected the C-ABI code object plus the team-kernel instances"
    assert codeobj.calls(SO) == []


@pytest.mark.skipif(not codeobj.have_objdump(), reason="llvm-objdump not installed")
def test_checker_sees_a_real_call(tmp_path):
    """the checker itself: a tiny HIP library with a noinline device function is flagged"""
    import subprocess
    src = tmp_path / "call.hip"
    src.write_text(
        "#include <hip/hip_runtime.h>\n"
        "__device__ __attribute__((noinline)) float f(float x) { return x * x + 1.0f; }\n"
        "__global__ void k(float* p) { p[threadIdx.x] = f(p[threadIdx.x]); }\n")
    so = tmp_path / "libcall.so"
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-fPIC", "-shared", "-o", str(so),
                        str(src)], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("hipcc unavailable: " + r.stderr[-200:])
    found = codeobj.calls(str(so))
    assert any("s_swappc_b64" == i for _, _, i in found) and any("_Z1ff" in f for _, f, _ in found), found
