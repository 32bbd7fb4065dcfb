"""Builds the MI355X engine library in-tree (no JIT cache, so the .so travels with the repo).

    rapido_amd/_lib/libptls_mi355x.so  <- csrc/gcm_engine.hip (hipcc, --offload-arch=gfx950)
                                         + csrc/aead_slot.c, csrc/tls_records.c, csrc/record_layer.c,
                                           csrc/fault_journal.c (host C, gcc; the last against libhsa-runtime64)
                                         + a generated build-id object (ptls_mi355x_build_id)
    tests/cpp/_build/libkernel_model.so <- tests/cpp/kernel_model.cpp (host clang++, test only)
    tests/cpp/_build/libguard_alloc.so  <- tests/cpp/guard_alloc.c (gcc against libamdhip64: guard-paged device
                                           memory for the GPU read-bounds test, test only)
    scripts/_build/rl_stream            <- scripts/rl_stream.c (gcc, against the library: bench.py's host-to-host
                                           record-layer stream driver, a measurement tool)
    scripts/_build/liblds_ceiling.so    <- scripts/lds_ceiling.hip (hipcc, build_lds_probe: the LDS-ceiling probe of
                                           scripts/gpu_lds_ceiling.sh, a measurement tool)

The library is stamped with a hash of its sources (source_build_id: rapido_amd/csrc/* and include/ptls_mi355x.h).
It is rebuilt from scratch whenever the stamp differs from the tree's hash, whatever the file times say, so the
.so that travels to the GPU box is the one HEAD's sources make; ptls_mi355x_build_id() returns the stamp.
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "_lib")
OBJDIR = os.path.join(PKG, "_lib", "obj")
LIB = os.path.join(LIBDIR, "libptls_mi355x.so")
STAMP = LIB + ".build_id"
HEADER = os.path.join(ROOT, "include", "ptls_mi355x.h")
MODEL_SRC = os.path.join(ROOT, "tests", "cpp", "kernel_model.cpp")
MODEL_LIB = os.path.join(ROOT, "tests", "cpp", "_build", "libkernel_model.so")
ARCH = os.environ.get("PTLS_MI355X_ARCH", "gfx950")

HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
CLANGXX = "/opt/rocm/llvm/bin/clang++" if os.path.exists("/opt/rocm/llvm/bin/clang++") else (shutil.which("clang++") or "clang++")
CC = shutil.which("gcc") or "cc"

HEADERS = [os.path.join(CSRC, "gcm_core.h"), HEADER]
# the VALU-engine measurement headers (scripts/) built only into the host model of the CPU test suite
MODEL_HEADERS = HEADERS + [os.path.join(ROOT, "scripts", "gcm_sbox.h"), os.path.join(ROOT, "scripts", "gcm_bitslice.h")]


def source_files():
    """The files the library is built from, in hash order: every regular file of csrc/, then the ABI header."""
    names = sorted(f for f in os.listdir(CSRC) if os.path.isfile(os.path.join(CSRC, f)))
    return [os.path.join(CSRC, f) for f in names] + [HEADER]


def source_build_id() -> str:
    """SHA-256 over "<name>\\0<bytes>" of source_files(), first 16 hex digits (ptls_mi355x_build_id)."""
    h = hashlib.sha256()
    for p in source_files():
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed: " + " ".join(cmd) + "\n" + r.stdout + r.stderr)
    return r


C_SRCS = [os.path.join(CSRC, f) for f in ("aead_slot.c", "tls_records.c", "record_layer.c", "fault_journal.c")]
ROCM_INCLUDE = "/opt/rocm/include"
C_OBJS = [os.path.join(OBJDIR, os.path.basename(f)[:-2] + ".o") for f in C_SRCS]
C_FLAGS = ["-std=gnu99", "-O2", "-g", "-fPIC", "-Wall", "-Wextra", "-Wno-unused-parameter", "-D__HIP_PLATFORM_AMD__",
           "-I" + ROCM_INCLUDE]


def stamped_build_id():
    """The build id the library in the tree was stamped with, or None."""
    try:
        with open(STAMP) as f:
            return f.read().strip() or None
    except OSError:
        return None


def build_engine(verbose: bool = False, force: bool = False) -> str:
    os.makedirs(OBJDIR, exist_ok=True)
    bid = source_build_id()
    # a stamp that differs from the sources' hash (or none) rebuilds every object, whatever the mtimes say
    force = force or stamped_build_id() != bid or not os.path.exists(LIB)
    hip_src = os.path.join(CSRC, "gcm_engine.hip")
    hip_obj = os.path.join(OBJDIR, "gcm_engine.o")
    if force or _newer(hip_obj, [hip_src] + HEADERS):
        _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-c", hip_src, "-o", hip_obj],
             verbose)
    for c_src, c_obj in zip(C_SRCS, C_OBJS):
        if force or _newer(c_obj, [c_src] + HEADERS):
            _run([CC] + C_FLAGS + ["-c", c_src, "-o", c_obj], verbose)
    bid_src = os.path.join(OBJDIR, "build_id.c")
    bid_obj = os.path.join(OBJDIR, "build_id.o")
    with open(bid_src, "w") as f:
        f.write("/* generated by rapido_amd/build.py: SHA-256 prefix of the library's sources */\n"
                f'const char *ptls_mi355x_build_id(void) {{ return "{bid}"; }}\n')
    _run([CC] + C_FLAGS + ["-c", bid_src, "-o", bid_obj], verbose)
    if force or _newer(LIB, [hip_obj] + C_OBJS):
        if os.path.exists(STAMP):
            os.remove(STAMP)
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, hip_obj, bid_obj] + C_OBJS +
             ["-L/opt/rocm/lib", "-lhsa-runtime64"], verbose)
        with open(STAMP, "w") as f:
            f.write(bid + "\n")
    return LIB


def build_model(verbose: bool = False, force: bool = False) -> str:
    """Host build of the kernel code for the CPU test suite (not part of the product)."""
    os.makedirs(os.path.dirname(MODEL_LIB), exist_ok=True)
    if force or _newer(MODEL_LIB, [MODEL_SRC] + MODEL_HEADERS):
        _run([CLANGXX, "-std=c++17", "-O2", "-fPIC", "-shared", "-Wall", "-o", MODEL_LIB, MODEL_SRC], verbose)
    return MODEL_LIB


GUARD_SRC = os.path.join(ROOT, "tests", "cpp", "guard_alloc.c")
GUARD_LIB = os.path.join(ROOT, "tests", "cpp", "_build", "libguard_alloc.so")


def build_guard(verbose: bool = False, force: bool = False) -> str:
    """Device memory with unmapped guard ranges (HIP virtual memory), for tests/test_gpu_read_bounds.py (test only)."""
    os.makedirs(os.path.dirname(GUARD_LIB), exist_ok=True)
    if force or _newer(GUARD_LIB, [GUARD_SRC]):
        _run([CC] + C_FLAGS + ["-shared", "-o", GUARD_LIB, GUARD_SRC, "-L/opt/rocm/lib", "-lamdhip64"], verbose)
    return GUARD_LIB


RL_STREAM_SRC = os.path.join(ROOT, "scripts", "rl_stream.c")
RL_STREAM = os.path.join(ROOT, "scripts", "_build", "rl_stream")


def build_rl_stream(verbose: bool = False, force: bool = False) -> str:
    """The C driver of bench.py's record_layer_stream (measurement, not part of the product)."""
    os.makedirs(os.path.dirname(RL_STREAM), exist_ok=True)
    if force or _newer(RL_STREAM, [RL_STREAM_SRC, LIB] + HEADERS):
        _run([CC, "-std=gnu99", "-O2", "-g", "-rdynamic", "-Wall", "-o", RL_STREAM, RL_STREAM_SRC, "-L" + LIBDIR, "-lptls_mi355x",
              "-Wl,-rpath,$ORIGIN/../../rapido_amd/_lib"], verbose)
    return RL_STREAM


LDS_PROBE_SRC = os.path.join(ROOT, "scripts", "lds_ceiling.hip")
LDS_PROBE = os.path.join(ROOT, "scripts", "_build", "liblds_ceiling.so")


def build_lds_probe(verbose: bool = False, force: bool = False) -> str:
    """The LDS-ceiling probe bench.py runs beside the batch kernels (measurement, not part of the product)."""
    os.makedirs(os.path.dirname(LDS_PROBE), exist_ok=True)
    if force or _newer(LDS_PROBE, [LDS_PROBE_SRC]):
        _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", LDS_PROBE_SRC, "-o", LDS_PROBE],
             verbose)
    return LDS_PROBE


def build_all(verbose: bool = False, force: bool = False) -> None:
    build_engine(verbose, force)
    build_model(verbose, force)
    build_guard(verbose, force)
    build_rl_stream(verbose, force)


if __name__ == "__main__":
    build_all(verbose=True, force="--force" in sys.argv)
    print(LIB, stamped_build_id())
