"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer.

SURVEY.md section 5 (race detection / sanitizers): the reference builds
with HPX_WITH_SANITIZERS (CMakeLists.txt:844,1732-1733); here the checker
itself -- oracle/oracle.cpp, host code -- is compiled with
-fsanitize=address,undefined -fno-sanitize-recover=all and driven over every
exported function at small and ragged sizes (tests/cxx/oracle_sanitize.cpp),
so an out-of-bounds access, leak or undefined operation in the oracle fails
this test instead of silently corrupting a parity reference.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("make") is None, reason="needs g++ and make")
def test_oracle_under_asan_ubsan():
    b = subprocess.run(["make", "-s", "oracle-sanitize"], cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert b.returncode == 0, b.stdout + b.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(ROOT, "tests/cxx/bin/oracle_sanitize")], cwd=ROOT, capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout
