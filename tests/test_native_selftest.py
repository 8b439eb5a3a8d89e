"""Native self-test executable (csrc/tests/native_selftest.cpp), plain and under host
AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5 race detection / sanitizers).

CPU: builds both variants for gfx950 and runs the host-only checks (ABI, planning, argument
validation) under the sanitizers. GPU: runs the full self-test (Gram, inverses, graph engine,
per-worker and blocked persistent kernels, first-order engine vs a host double reference)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

ASAN_ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
                UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _exe(asan):
    import build_selftest

    return build_selftest.build(asan=asan, jobs=8, verbose=False)


@pytest.mark.parametrize("asan", [False, True])
def test_selftest_host_only(asan):
    exe = _exe(asan)
    env = dict(ASAN_ENV, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1") if asan else None
    r = subprocess.run([exe, "--host-only"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "native_selftest: OK" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("asan", [False, True])
def test_selftest_gpu(asan):
    exe = _exe(asan)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=ASAN_ENV if asan else None)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "native_selftest: OK (host + GPU)" in r.stdout
