"""ASan + UBSan run of the path's host-side C++ (SURVEY.md §5 "Race detection /
sanitizers"): the oracle restatement and the product's host IRLS /
decomposition (csrc/host_polish.cpp) built with -fsanitize=address,undefined
-fno-sanitize-recover=all (oracle/Makefile `sanitize`) and driven over
ordinary, degenerate and edge inputs by oracle/sanitize/driver.cpp.  Any
memory error, leak or undefined behaviour aborts the driver with a report."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_code_is_sanitizer_clean():
    subprocess.run(["make", "-s", "-B", "-C", os.path.join(ROOT, "oracle"), "sanitize"], check=True,
                   capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1",
               OMP_NUM_THREADS="1")
    r = subprocess.run([os.path.join(ROOT, "oracle", "_san", "sanitize_driver")], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "sanitize ok" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
