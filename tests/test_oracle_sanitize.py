"""The CPU oracle (the repo's only physics truth, SURVEY.md §5 "Race detection / sanitizers") under
AddressSanitizer + UndefinedBehaviorSanitizer: `make -C oracle sanitize` builds build_san/liboracle_san.so and the
oracle test files run against it in a child python with the sanitizer runtimes preloaded (host code only; the
GPU pool has no device sanitizers).  Any heap/stack overflow, use-after-free or UB aborts the child."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


def _runtime(name):
    p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.mark.timeout(900)
def test_oracle_tests_clean_under_asan_ubsan():
    asan, ubsan = _runtime("libasan.so"), _runtime("libubsan.so")
    if not (asan and ubsan):
        pytest.skip("gcc sanitizer runtimes not installed")
    subprocess.check_call(["make", "-s", "-C", ORACLE, "sanitize"])
    lib = os.path.join(ORACLE, "build_san", "liboracle_san.so")
    env = dict(os.environ, MG_ORACLE_LIB=lib, LD_PRELOAD=f"{asan}:{ubsan}",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    files = ["test_oracle_physics.py", "test_oracle_hand_physics.py", "test_oracle_golden.py", "test_dr.py"]
    # the child asserts it really loaded the sanitizer build before running the oracle tests
    code = ("import sys, ctypes; sys.path.insert(0, %r); import pyoracle; assert pyoracle.LIB == %r; "
            "pyoracle.lib(); import pytest; sys.exit(pytest.main(['-q', '-x', '-p', 'no:cacheprovider', "
            "'-m', 'not gpu'] + %r))") % (ORACLE, lib, [os.path.join(ROOT, "tests", f) for f in files])
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    assert "passed" in r.stdout and "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, tail
