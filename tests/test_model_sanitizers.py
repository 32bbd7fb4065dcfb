"""The host kernel model under AddressSanitizer + UndefinedBehaviorSanitizer (CPU, deterministic).

tests/cpp/model_sanitize.cpp drives every kernel family's code path of gcm_core.h (batch K = 1, 2, 4, 8; window 4/8
lanes, 64/32-position segments; 16-lane; split; TLS batch and window), AES-128 and AES-256, seal and open, on
exactly-sized heap buffers, with the walk's reads and stores held to each record's bytes (GCM_READ / GCM_WRITE).  Built
with -fsanitize=address,undefined as its own executable (sanitizers on host code only), so an access outside the
emulated LDS image, the key image, the tables or a stack array, or undefined behaviour in the kernel code's host
compile, fails here."""
import os
import subprocess

import pytest

from rapido_amd import build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "model_sanitize.cpp")
EXE = os.path.join(ROOT, "tests", "cpp", "_build", "model_sanitize")
DEPS = [SRC, build.MODEL_SRC] + build.MODEL_HEADERS


def _build():
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    if os.path.exists(EXE) and all(os.path.getmtime(d) <= os.path.getmtime(EXE) for d in DEPS):
        return EXE
    r = subprocess.run([build.CLANGXX, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                        "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-o", EXE, SRC],
                       capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        pytest.fail("sanitizer build failed:\n" + r.stderr[-4000:])
    return EXE


def test_kernel_model_is_clean_under_asan_and_ubsan():
    exe = _build()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-6000:]
    assert "model_sanitize: ok (0 failures" in out, out[-2000:]
    assert "AddressSanitizer" not in out and "runtime error" not in out, out[-6000:]
