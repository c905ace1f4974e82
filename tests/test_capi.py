"""The C-ABI library loads on a GPU-less host and exports every function
include/scann_mi355x.h declares; argument validation that happens before any
HIP call is exercised here (no device work)."""
import ctypes
import os
import re

import numpy as np
import pytest

from tests.conftest import ROOT

HEADER = os.path.join(ROOT, "include", "scann_mi355x.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(smx_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    from scann_amd import build
    build.build()
    from scann_amd import _native
    return _native.load()


def test_header_declares_the_boundary():
    fns = declared_functions()
    for f in ("smx_index_create", "smx_search_batched", "smx_index_destroy", "smx_last_error"):
        assert f in fns


def test_library_exports_every_declared_symbol(lib):
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing


def test_library_resolves_every_internal_symbol(lib):
    """A lazily bound load hides a missing definition until the first call:
    every symbol of the library's own namespace must be defined in it."""
    from scann_amd import build
    out = os.popen(f"nm -D --undefined-only {build.OUT}").read()
    assert "_ZN3smx" not in out, [l for l in out.splitlines() if "_ZN3smx" in l]
    ctypes.CDLL(build.OUT, mode=os.RTLD_NOW | os.RTLD_LOCAL)


def test_binding_covers_every_declared_symbol():
    from scann_amd import _native
    assert sorted(_native.SIGNATURES) == declared_functions()


def test_version_and_error_reporting_without_gpu(lib):
    assert b"gfx950" in lib.smx_version()
    from scann_amd import _native
    h = ctypes.c_void_p()
    rc = lib.smx_index_create(None, 0, ctypes.byref(h))
    assert rc == -1 and b"null index description" in lib.smx_last_error()


def test_descriptor_validation_without_gpu(lib, small_dot):
    from scann_amd import _native
    ix = small_dot[0]
    d = ix.desc()
    d.num_blocks = 65
    h = ctypes.c_void_p()
    assert lib.smx_index_create(ctypes.byref(d), 0, ctypes.byref(h)) == -1
    assert b"at most 64" in lib.smx_last_error()
    d = ix.desc()
    d.dims_per_block = 1  # 16 blocks x 1 dim do not tile 32 dims
    assert lib.smx_index_create(ctypes.byref(d), 0, ctypes.byref(h)) == -1
    bad = ix.member_codes.copy()
    bad[0, 0] = 16
    d = ix.desc()
    d.member_codes = bad.ctypes.data
    assert lib.smx_index_create(ctypes.byref(d), 0, ctypes.byref(h)) == -1
    assert b"< 16" in lib.smx_last_error()
    p = _native.SearchParams(0, 10, 10, 1)
    assert lib.smx_search_batched(None, None, 0, 32, ctypes.byref(p), None, None, None) == -1


def test_struct_layout_matches_header(tmp_path):
    """IndexDesc / SearchParams / Timings (ctypes) mirror the header: every
    field offset and the struct sizes, as the C compiler lays them out."""
    import os
    import subprocess
    from scann_amd.index import IndexDesc
    from scann_amd._native import SearchParams, Timings
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    structs = {"smx_index_desc": IndexDesc, "smx_search_params": SearchParams,
               "smx_timings": Timings}
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "scann_mi355x.h"',
             "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'  printf("{cname} %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            cf = "reserved" if (cname == "smx_index_desc" and fname == "pad_") else fname
            lines.append(f'  printf("{cname}.{fname} %zu\\n", offsetof({cname}, {cf}));')
    lines.append('  printf("smx_shard_entry %zu\\n", sizeof(smx_shard_entry));')
    lines.append("  return 0;\n}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(root, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], check=True, capture_output=True,
                                                         text=True).stdout.splitlines())
    for cname, py in structs.items():
        assert int(got[cname]) == ctypes.sizeof(py), cname
        for fname, _ in py._fields_:
            assert int(got[f"{cname}.{fname}"]) == getattr(py, fname).offset, (cname, fname)
    assert int(got["smx_shard_entry"]) == 16


def test_pybind_module_surface():
    """The C++ pybind11 module (scann_amd/csrc/smx_pybind.cc) loads and has the
    reference's ScannNumpy search surface (scann_pybind.cc:24-54); no GPU
    call is made here."""
    from scann_amd import _native
    mod = _native.load_pybind()
    core = mod.ScannNumpyCore
    for name in ("search", "search_batched", "size", "dim"):
        assert callable(getattr(core, name))
    doc = core.search_batched.__doc__
    assert "queries" in doc and "parallel" in doc and "batch_size" in doc
    with pytest.raises(ValueError, match="null index description"):
        core(0, 0, 10, 100, 100, True, True)
