"""Host-runtime sanitizer builds: csrc/runtime/*.cpp compiled with -fsanitize=address / thread /
undefined into the self-test driver csrc/runtime/tests/selftest.cpp (ops/build.py --sanitize=...), which exercises
every runtime entry point, multi-threaded where the runtime is; a sanitizer report or a wrong result fails."""
import os
import shutil
import subprocess

import pytest

from deeplearning4j_amd.ops.build import SANITIZERS, build_runtime_sanitized


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
@pytest.mark.parametrize("kind", SANITIZERS)
def test_runtime_selftest_under_sanitizer(kind):
    exe = build_runtime_sanitized(kind, verbose=False)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1", TSAN_OPTIONS="halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "runtime selftest OK" in r.stdout
    assert "Sanitizer" not in r.stderr, r.stderr
