"""ASan + UBSan runs of the host-side C/C++ (CPU only, no GPU needed).

Builds ``tests/native/Makefile`` into ``oracle/_ref/san`` and runs each driver:

* ``san_oracle``   every oracle entry point over edge shapes and values
  (L = 1, ragged tails, K < L, NaN/inf, n_grid = 1, empty batches);
* ``san_planners`` the library's host planners (ragged/table planners,
  the stream batch planner) and their error paths.  Device code is not
  instrumented (``-fno-gpu-sanitize``; GPU ASan is unavailable on this pool);
  no entry point that launches a kernel is called.

A sanitizer finding aborts the driver (``-fno-sanitize-recover=all``), so a
zero exit code plus the driver's "clean" line is the pass condition.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
OUT = os.path.join(ROOT, "oracle", "_ref", "san")

pytestmark = [
    pytest.mark.skipif(
        shutil.which("gcc") is None or not os.path.exists("/opt/rocm/bin/hipcc"),
        reason="sanitizer builds need gcc and hipcc"),
    # tests/native is listed in .gpurunignore: the GPU box gets no sanitizer sources.
    pytest.mark.skipif(not os.path.exists(os.path.join(NATIVE, "Makefile")),
                       reason="tests/native not shipped (GPU box snapshot)"),
]


def _build(target):
    r = subprocess.run(["make", "-s", "-C", NATIVE, f"OUT={OUT}", os.path.join(OUT, target)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    return os.path.join(OUT, target)


def _run(exe):
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0:halt_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-6000:]
    assert "clean" in out, out[-2000:]
    assert "runtime error" not in out and "AddressSanitizer" not in out, out[-6000:]
    return out


def test_oracle_under_asan_ubsan():
    _run(_build("san_oracle"))


def test_host_planners_under_asan_ubsan():
    _run(_build("san_planners"))
