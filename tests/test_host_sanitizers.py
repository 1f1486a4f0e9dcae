"""The library's host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only): the
host sources built with g++ -fsanitize=address,undefined and linked with the library's own HIP
objects into tests/native/build/host_asan, which fits through pc_fit_with_evaluator over C++
callbacks (tests/native/host_asan_driver.cpp): orthogonal screened and exact, non-orthogonal
multi-try (the convexity rejection) and per-try, extended, three densities, FastICA and JADE warm
starts. Any sanitizer report fails the run (UBSan without recovery; LeakSanitizer at exit)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBB = os.path.join(ROOT, "picard-ica_amd", "build")


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("make") is None, reason="no g++ / make")
def test_host_code_under_sanitizers():
    objs = [os.path.join(LIBB, f) for f in ("device.o", "screen.o", "collective.o")]
    if not all(os.path.exists(o) for o in objs):
        pytest.skip("library objects not built (make -C picard-ica_amd)")
    b = subprocess.run(["make", "-s", "-f", os.path.join(ROOT, "tests", "native", "Makefile.asan"), "-j4"],
                       capture_output=True, text=True, timeout=600)
    assert b.returncode == 0, b.stdout + b.stderr
    env = dict(os.environ, PICARD_TRACE="1", OMP_NUM_THREADS="4",
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(ROOT, "tests", "native", "build", "host_asan")], capture_output=True,
                       text=True, timeout=600, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "all fits ok" in r.stdout
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out and "LeakSanitizer" not in out
    # the rejection paths ran under the sanitizers
    assert "[picard-cvx]" in r.stderr and "[picard-curv]" in r.stderr and "[picard-screen]" in r.stderr
