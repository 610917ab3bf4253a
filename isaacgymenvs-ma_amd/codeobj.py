"""Static checks of the gfx950 code objects inside the built library (libmigym.so).

The team kernels must contain no real calls: every phase is force-inlined.  Round 3 saw a
real call into the narrowphase miscompile with this toolchain (wrong object states with IPRA on; an illegal
address and a 93 % parity build with IPRA off), and the inliner has declined a forceinline before (fk(),
DESIGN.md §3 Resources).  ``calls(so)`` lists every ``s_swappc_b64`` (a call) and ``s_setpc_b64 s[30:31]`` (a
return: only a callable function has one; long branches use s_setpc_b64 on other registers) in the device code, per code object, so build.py can fail
the build and tests/test_code_objects.py can assert on the shipped library.

The fat binary is read without the ROCm bundler: the ELF section ``.hip_fatbin`` holds one clang offload
bundle per translation unit ("__CLANG_OFFLOAD_BUNDLE__", entry count, then (offset, size, triple) per entry),
and the gfx950 entry of each is an AMDGPU ELF that ``llvm-objdump -d`` disassembles.
"""
import os
import re
import struct
import subprocess
import tempfile

def _objdump():
    """llvm-objdump of the ROCm install that builds the library: MIGYM_OBJDUMP, else <root>/lib/llvm/bin/llvm-objdump
    with <root> from ROCM_PATH, or from the hipcc in use (HIPCC, or hipcc on PATH: <root>/bin/hipcc), else /opt/rocm"""
    if os.environ.get("MIGYM_OBJDUMP"):
        return os.environ["MIGYM_OBJDUMP"]
    roots = []
    if os.environ.get("ROCM_PATH"):
        roots.append(os.environ["ROCM_PATH"])
    import shutil
    hipcc = os.environ.get("HIPCC") or shutil.which("hipcc")
    if hipcc:
        roots.append(os.path.dirname(os.path.dirname(os.path.realpath(hipcc))))
    roots.append("/opt/rocm")
    for r in roots:
        cand = os.path.join(r, "lib", "llvm", "bin", "llvm-objdump")
        if os.path.exists(cand):
            return cand
    raise FileNotFoundError("codeobj: no llvm-objdump under " + ", ".join(f"{r}/lib/llvm/bin" for r in roots) +
                            "; set MIGYM_OBJDUMP to its path (or ROCM_PATH to the ROCm root)")


def have_objdump():
    try:
        return os.path.exists(_objdump())
    except FileNotFoundError:
        return False


MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _section(path, name):
    d = open(path, "rb").read()
    if d[:4] != b"\x7fELF" or d[4] != 2:
        raise ValueError(f"{path}: not an ELF64 file")
    shoff, = struct.unpack_from("<Q", d, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", d, 0x3A)
    hdrs = [struct.unpack_from("<IIQQQQIIQQ", d, shoff + i * shentsize) for i in range(shnum)]
    strtab = hdrs[shstrndx]
    for h in hdrs:
        nm = d[strtab[4] + h[0]:d.index(b"\0", strtab[4] + h[0])].decode()
        if nm == name:
            return d[h[4]:h[4] + h[5]]
    raise ValueError(f"{path}: no {name} section")


def device_code_objects(so, arch="gfx950"):
    """the AMDGPU code objects (bytes) of every offload bundle in the library's .hip_fatbin"""
    fb = _section(so, ".hip_fatbin")
    out = []
    i = fb.find(MAGIC)
    while i >= 0:
        n, = struct.unpack_from("<Q", fb, i + len(MAGIC))
        p = i + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", fb, p)
            triple = fb[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if triple.startswith("hip") and triple.endswith(arch):
                out.append(fb[i + off:i + off + size])
        i = fb.find(MAGIC, i + 1)
    return out


def calls(so, arch="gfx950"):
    """[(code object index, function, instruction)] for every call / return in the device code"""
    found = []
    with tempfile.TemporaryDirectory() as td:
        for k, co in enumerate(device_code_objects(so, arch)):
            f = os.path.join(td, f"co{k}.o")
            with open(f, "wb") as fh:
                fh.write(co)
            txt = subprocess.run([_objdump(), "-d", f"--mcpu={arch}", f], capture_output=True, text=True,
                                 check=True).stdout
            fn = "?"
            for line in txt.splitlines():
                m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
                if m:
                    fn = m.group(1)
                elif "s_swappc_b64" in line or re.search(r"s_setpc_b64\s+s\[30:31\]", line):
                    # a call, or a return through the return address (s[30:31]): a callable function.  Long
                    # branches (s_getpc_b64 + add + s_setpc_b64 on other registers) are kernels' own jumps
                    found.append((k, fn, line.split()[0]))
    return found


def check_no_calls(so, arch="gfx950"):
    bad = calls(so, arch)
    if bad:
        fns = sorted({f for _, f, _ in bad})
        raise RuntimeError(f"{so}: the device code has real calls / returns (the team kernels must be fully "
                           f"inlined, DESIGN.md §3b): {fns[:8]}")
    return True
