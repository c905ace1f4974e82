"""Builds libscann_mi355x.so in-tree with hipcc for gfx950.

    python -m scann_amd.build
"""
from __future__ import annotations

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "scann_amd", "csrc")
OUT = os.path.join(ROOT, "scann_amd", "lib", "libscann_mi355x.so")
SOURCES = ["smx_kernels.hip", "smx_searcher.hip", "smx_builder.hip", "smx_sort.hip"]
HEADERS = ["smx_internal.h", os.path.join("..", "..", "include", "scann_mi355x.h")]
ARCH = os.environ.get("SMX_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in (os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc"), "hipcc"):
        if os.path.sep not in c or os.path.exists(c):
            return c
    return "hipcc"


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.abspath(__file__)]
    return any(os.path.getmtime(p) > t for p in deps if os.path.exists(p))


def build(force: bool = False, verbose: bool = False, defines=(), out: str = OUT) -> str:
    """The product library; `defines` + `out` make a diagnostic variant
    (e.g. ("SMX_PHASE_STAMPS",) -> lib/libscann_mi355x_ps.so, loaded through
    $SMX_LIB by the tools only)."""
    if not force and out == OUT and not needs_build():
        return OUT
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tmp = out + f".tmp{os.getpid()}"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-ffp-contract=off", "-Wall", "-o", tmp] + [f"-D{d}" for d in defines] + \
        [os.path.join(CSRC, f) for f in SOURCES]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out


PYBIND_SRC = os.path.join(CSRC, "smx_pybind.cc")


def pybind_path() -> str:
    import sysconfig
    return os.path.join(os.path.dirname(OUT), "_smx_pybind" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_pybind(force: bool = False, verbose: bool = False) -> str:
    """The C++ pybind11 module (scann_amd/csrc/smx_pybind.cc) over the C ABI,
    next to the library it links (rpath $ORIGIN)."""
    import sysconfig

    import pybind11
    out = pybind_path()
    deps = [PYBIND_SRC, OUT, os.path.join(ROOT, "include", "scann_mi355x.h")]
    if not force and os.path.exists(out) and all(
            os.path.getmtime(out) >= os.path.getmtime(d) for d in deps if os.path.exists(d)):
        return out
    tmp = out + f".tmp{os.getpid()}"
    cmd = ["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-Wall", "-fvisibility=hidden",
           f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}", PYBIND_SRC,
           f"-L{os.path.dirname(OUT)}", "-l:libscann_mi355x.so", "-Wl,-rpath,$ORIGIN", "-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out


DIAG_OUT = os.path.join(ROOT, "scann_amd", "lib", "libscann_mi355x_diag.so")
# The diagnostic library (loaded through $SMX_LIB by tools/ and by the
# debug-check test run only): device index checks on every computed index
# (a violation fails the call with SMX_INTERNAL), the scan's timing
# ablations and per-segment stamps, and the front-end/select phase stamps.
DIAG_DEFINES = ("SMX_DEBUG_CHECKS", "SMX_SCAN_DIAGNOSTICS", "SMX_PHASE_STAMPS")


TIME_OUT = os.path.join(ROOT, "scann_amd", "lib", "libscann_mi355x_time.so")
# The timing library: the scan ablations/stamps and the phase stamps without
# the device index checks (whose extra registers and branches change the
# kernels' occupancy and timing); loaded through $SMX_LIB by tools/ only.
TIME_DEFINES = ("SMX_SCAN_DIAGNOSTICS", "SMX_PHASE_STAMPS")


def build_time(force: bool = False, verbose: bool = False) -> str:
    if not force and os.path.exists(TIME_OUT) and not needs_build_for(TIME_OUT):
        return TIME_OUT
    return build(force=True, verbose=verbose, defines=TIME_DEFINES, out=TIME_OUT)


def build_diag(force: bool = False, verbose: bool = False) -> str:
    if not force and os.path.exists(DIAG_OUT) and not needs_build_for(DIAG_OUT):
        return DIAG_OUT
    return build(force=True, verbose=verbose, defines=DIAG_DEFINES, out=DIAG_OUT)


def needs_build_for(out: str) -> bool:
    t = os.path.getmtime(out)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.abspath(__file__)]
    return any(os.path.getmtime(p) > t for p in deps if os.path.exists(p))


if __name__ == "__main__":
    if "--diag" in sys.argv:
        print(build_diag(force="--force" in sys.argv, verbose=True))
        sys.exit(0)
    if "--time" in sys.argv:
        print(build_time(force="--force" in sys.argv, verbose=True))
        sys.exit(0)
    print(build(force="--force" in sys.argv, verbose=True))
    print(build_pybind(force="--force" in sys.argv, verbose=True))
