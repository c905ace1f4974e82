"""ctypes binding of libscann_mi355x.so (include/scann_mi355x.h).

This is the reference-side binding a maintainer would add in place of the
``scann_pybind`` extension (scann/scann_ops/cc/python/scann_pybind.cc).
There is no CPU fallback: if the library is missing or fails to load, import
raises, and every search runs the HIP kernels.
"""
from __future__ import annotations

import ctypes
import sys
import os

import numpy as np

from .index import IndexDesc

_HERE = os.path.dirname(os.path.abspath(__file__))
# SMX_LIB: an alternative build of the same library (tuning experiments)
PRODUCT_LIB = os.path.join(_HERE, "lib", "libscann_mi355x.so")
LIB_PATH = os.environ.get("SMX_LIB") or PRODUCT_LIB

SMX_OK = 0


class SearchParams(ctypes.Structure):
    _fields_ = [("leaves_to_search", ctypes.c_int32), ("pre_reorder_nn", ctypes.c_int32),
                ("final_nn", ctypes.c_int32), ("reorder", ctypes.c_int32)]


class Timings(ctypes.Structure):
    _fields_ = [("partition_ms", ctypes.c_float), ("lut_ms", ctypes.c_float),
                ("invert_ms", ctypes.c_float), ("seed_scan_ms", ctypes.c_float),
                ("seed_select_ms", ctypes.c_float), ("scan_ms", ctypes.c_float),
                ("select_ms", ctypes.c_float), ("total_ms", ctypes.c_float),
                ("scan_code_bytes", ctypes.c_double), ("seed_code_bytes", ctypes.c_double),
                ("scan_pairs", ctypes.c_int32), ("seed_pairs", ctypes.c_int32),
                ("overflow_retries", ctypes.c_int32), ("max_candidates", ctypes.c_int32),
                ("scan_item_tiles", ctypes.c_double), ("mean_candidates", ctypes.c_float),
                ("scan_workgroups", ctypes.c_int32), ("scan_item_tiles16", ctypes.c_double),
                ("scan_launches", ctypes.c_int32), ("scan_ms_mode2", ctypes.c_float)]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


# name -> (restype, argtypes); must cover every function of include/scann_mi355x.h
_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
SIGNATURES = {
    "smx_index_create": (ctypes.c_int, [ctypes.POINTER(IndexDesc), _i32, ctypes.POINTER(_vp)]),
    "smx_index_destroy": (ctypes.c_int, [_vp]),
    "smx_index_info": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp]),
    "smx_search_batched": (ctypes.c_int, [_vp, _vp, _i32, _i32, ctypes.POINTER(SearchParams), _vp, _vp, _vp]),
    "smx_search": (ctypes.c_int, [_vp, _vp, _i32, ctypes.POINTER(SearchParams), _vp, _vp, _vp]),
    "smx_search_batched_device": (ctypes.c_int, [_vp, _vp, _i32, _i32, ctypes.POINTER(SearchParams), _vp, _vp, _vp, _vp]),
    "smx_partition_topl": (ctypes.c_int, [_vp, _vp, _i32, _i32, _vp, _vp]),
    "smx_create_lookup_tables": (ctypes.c_int, [_vp, _vp, _i32, _vp, _vp]),
    "smx_search_pre_reorder": (ctypes.c_int, [_vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp]),
    "smx_exact_distances": (ctypes.c_int, [_vp, _vp, _i32, _vp, _i32, _vp]),
    "smx_lut16_leaf_scores": (ctypes.c_int, [_vp, _i32, _vp, _vp]),
    "smx_kth_threshold_keys": (ctypes.c_int, [_vp, _i32, _i32, _vp, _vp]),
    "smx_set_profiling": (ctypes.c_int, [_vp, _i32]),
    "smx_release_stream": (ctypes.c_int, [_vp, _vp]),
    "smx_get_timings": (ctypes.c_int, [_vp, ctypes.POINTER(Timings)]),
    "smx_set_tuning": (ctypes.c_int, [_vp, _i32, _i32, _i32, _i32]),
    "smx_shard_width": (ctypes.c_int, [_vp, ctypes.POINTER(SearchParams), ctypes.POINTER(_i32)]),
    "smx_search_shard_device": (ctypes.c_int, [_vp, _vp, _i32, _i32, ctypes.POINTER(SearchParams), _vp, _vp]),
    "smx_merge_shards_device": (ctypes.c_int, [_vp, _i32, _i32, ctypes.POINTER(SearchParams), _vp, _vp, _vp, _vp, _vp]),
    "smx_nearest_centers": (ctypes.c_int, [_vp, ctypes.c_int64, _i32, _vp, _i32, _vp,
                                           ctypes.c_float, _vp, _vp, _vp]),
    "smx_block_encode": (ctypes.c_int, [_vp, ctypes.c_int64, _i32, _vp, _i32, _i32, _vp, _vp]),
    "smx_avq_encode": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _i32, _vp, _i32, _i32,
                                      ctypes.c_double, _vp, _vp]),
    "smx_kmeans_accumulate": (ctypes.c_int, [_vp, ctypes.c_int64, _i32, _vp, _i32,
                                             ctypes.c_double, _vp, _vp, _vp]),
    "smx_kmeans_finalize": (ctypes.c_int, [_vp, _vp, _i32, _i32, ctypes.c_double, _vp, _vp]),
    "smx_codebook_accumulate": (ctypes.c_int, [_vp, ctypes.c_int64, _i32, _vp, _i32, _i32,
                                               ctypes.c_double, _vp, _vp, _vp]),
    "smx_group_by_leaf": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _i32, _vp,
                                         ctypes.POINTER(ctypes.c_size_t), _vp, _vp, _vp, _vp,
                                         _vp]),
    "smx_gather_residuals": (ctypes.c_int, [_vp, _i32, _vp, _vp, _vp, ctypes.c_int64,
                                            ctypes.c_int64, _vp, _vp]),
    "smx_last_error": (ctypes.c_char_p, []),
    "smx_version": (ctypes.c_char_p, []),
}

_lib = None


def load(path: str = LIB_PATH):
    """Load the HIP library; raises ImportError (loudly) if it is unusable."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(
            f"{path} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (the MI355X search path has no CPU fallback)")
    # torch first: it brings its own HIP/HSA runtime, which the library then
    # binds by soname.  Loaded the other way round, /opt/rocm's runtime comes
    # in first and torch's later device init fails ("No HIP GPUs are
    # available") -- one process, one runtime (load order).
    # Without torch the library binds /opt/rocm's runtime by itself.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        # a library built from an older source (an A/B of $SMX_LIB builds)
        # may predate an entry point: it then fails when called, not here;
        # the product library exports every one (tests/test_capi.py)
        fn = getattr(lib, name, None)
        if fn is None and os.path.abspath(path) == PRODUCT_LIB:
            raise ImportError(f"{path} does not export {name}: rebuild it")
        if fn is not None:
            fn.restype = res
            fn.argtypes = args
    _lib = lib
    return lib


_pybind = None


def load_pybind():
    """The C++ pybind11 module (ScannNumpyCore, scann_amd/csrc/smx_pybind.cc);
    raises ImportError (loudly) if it was not built."""
    global _pybind
    if _pybind is not None:
        return _pybind
    import importlib.machinery
    import importlib.util
    import sysconfig
    path = os.path.join(_HERE, "lib", "_smx_pybind" + sysconfig.get_config_var("EXT_SUFFIX"))
    if not os.path.exists(path):
        raise ImportError(f"{path} not found: build it with `python -m scann_amd.build`")
    loader = importlib.machinery.ExtensionFileLoader("_smx_pybind", path)
    spec = importlib.util.spec_from_file_location("_smx_pybind", path, loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    _pybind = mod
    return mod


class SmxError(RuntimeError):
    pass


def check(rc: int, what: str) -> None:
    if rc != SMX_OK:
        msg = load().smx_last_error().decode(errors="replace")
        raise SmxError(f"{what}: {msg} (status {rc})")


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def _current_stream(stream):
    """The HIP stream a device entry point runs on: the caller's, else torch's
    current stream when torch is in use (the device entry points return with
    the work enqueued, so results are ordered with the caller's own reads and
    writes of those buffers), else the library's own stream (None)."""
    if stream is not None:
        return stream
    torch = sys.modules.get("torch")
    if torch is not None and torch.cuda.is_available() and torch.cuda.is_initialized():
        return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    return None


def kth_threshold_keys_device(vals_ptr, sets, kk, out_ptr, stream=None):
    """smx_kth_threshold_keys on device buffers (the seed threshold select)."""
    check(load().smx_kth_threshold_keys(vals_ptr, int(sets), int(kk), out_ptr, stream),
          "smx_kth_threshold_keys")


def nearest_centers_device(x_ptr, n, d, c_ptr, k, out_ptr, primary_ptr=None, lam=0.0,
                           loss_ptr=None, stream=None):
    """smx_nearest_centers on device buffers (k-means / SOAR assignment)."""
    check(load().smx_nearest_centers(x_ptr, int(n), int(d), c_ptr, int(k), primary_ptr,
                                     float(lam), out_ptr, loss_ptr, _current_stream(stream)),
          "smx_nearest_centers")


class NativeIndex:
    """Owns one smx_index handle (device-resident index)."""

    def __init__(self, index, device: int = 0):
        self.lib = load()
        self.index = index
        self.dim = index.dim
        desc = index.desc()
        h = _vp()
        check(self.lib.smx_index_create(ctypes.byref(desc), device, ctypes.byref(h)),
              "smx_index_create")
        self.h = h

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.lib.smx_index_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self):
        d, l, s = _i32(), _i32(), _i32()
        n = ctypes.c_uint32()
        check(self.lib.smx_index_info(self.h, ctypes.byref(d), ctypes.byref(l), ctypes.byref(n),
                                      ctypes.byref(s)), "smx_index_info")
        return dict(dim=d.value, num_leaves=l.value, num_datapoints=n.value,
                    global_topn_shift=s.value)

    def search_batched(self, queries, leaves, pre_nn, final_nn, reorder=True):
        q = _c(queries, np.float32)
        if q.ndim != 2:
            raise ValueError("Queries must be in two-dimensional array")
        nq = q.shape[0]
        p = SearchParams(int(leaves), int(pre_nn), int(final_nn), int(bool(reorder)))
        idx = np.zeros((nq, final_nn), np.uint32)
        dist = np.zeros((nq, final_nn), np.float32)
        cnt = np.zeros(nq, np.int32)
        check(self.lib.smx_search_batched(self.h, q.ctypes.data, nq, q.shape[1], ctypes.byref(p),
                                          idx.ctypes.data, dist.ctypes.data, cnt.ctypes.data),
              "Error during search")
        return idx, dist, cnt

    def search(self, query, leaves, pre_nn, final_nn, reorder=True):
        """One query through the single-query numerics (smx_search)."""
        q = _c(query, np.float32)
        if q.ndim != 1:
            raise ValueError("Query must be one-dimensional")
        p = SearchParams(int(leaves), int(pre_nn), int(final_nn), int(bool(reorder)))
        idx = np.zeros(final_nn, np.uint32)
        dist = np.zeros(final_nn, np.float32)
        cnt = np.zeros(1, np.int32)
        check(self.lib.smx_search(self.h, q.ctypes.data, q.shape[0], ctypes.byref(p),
                                  idx.ctypes.data, dist.ctypes.data, cnt.ctypes.data),
              "Error during search")
        return idx, dist, int(cnt[0])

    def search_batched_device(self, q_ptr, nq, leaves, pre_nn, final_nn, reorder,
                              out_idx_ptr, out_dist_ptr, out_count_ptr=None, stream=None):
        p = SearchParams(int(leaves), int(pre_nn), int(final_nn), int(bool(reorder)))
        check(self.lib.smx_search_batched_device(self.h, q_ptr, nq, self.dim, ctypes.byref(p),
                                                 out_idx_ptr, out_dist_ptr, out_count_ptr,
                                                 _current_stream(stream)),
              "Error during search")

    def release_stream(self, stream=None):
        """Waits for this handle's work on `stream` and frees its workspace
        (smx_release_stream): the stream may then be destroyed."""
        check(self.lib.smx_release_stream(self.h, _current_stream(stream)), "smx_release_stream")

    # -- range-split shards; device pointers ----------------
    SHARD_ENTRY_BYTES = 16   # smx_shard_entry {u64 key; u32 id; f32 exact}

    def shard_width(self, leaves, pre_nn, final_nn, reorder=True) -> int:
        p = SearchParams(int(leaves), int(pre_nn), int(final_nn), int(bool(reorder)))
        k = _i32()
        check(self.lib.smx_shard_width(self.h, ctypes.byref(p), ctypes.byref(k)), "smx_shard_width")
        return k.value

    def search_shard_device(self, q_ptr, nq, leaves, pre_nn, final_nn, reorder, entries_ptr,
                            stream=None):
        p = SearchParams(int(leaves), int(pre_nn), int(final_nn), int(bool(reorder)))
        check(self.lib.smx_search_shard_device(self.h, q_ptr, nq, self.dim, ctypes.byref(p),
                                               entries_ptr, _current_stream(stream)),
              "Error during search")

    def merge_shards_device(self, world, nq, leaves, pre_nn, final_nn, reorder, entries_ptr,
                            out_idx_ptr, out_dist_ptr, out_count_ptr=None, stream=None):
        p = SearchParams(int(leaves), int(pre_nn), int(final_nn), int(bool(reorder)))
        check(self.lib.smx_merge_shards_device(self.h, int(world), int(nq), ctypes.byref(p),
                                               entries_ptr, out_idx_ptr, out_dist_ptr,
                                               out_count_ptr, _current_stream(stream)),
              "smx_merge_shards")

    def search_pre_reorder(self, queries, leaves, pre_nn):
        q = _c(queries, np.float32)
        nq = q.shape[0]
        idx = np.zeros((nq, pre_nn), np.uint32)
        dist = np.zeros((nq, pre_nn), np.float32)
        cnt = np.zeros(nq, np.int32)
        check(self.lib.smx_search_pre_reorder(self.h, q.ctypes.data, nq, leaves, pre_nn,
                                              idx.ctypes.data, dist.ctypes.data, cnt.ctypes.data),
              "smx_search_pre_reorder")
        return idx, dist, cnt

    def partition_topl(self, queries, L):
        q = _c(queries, np.float32)
        leaf = np.zeros((q.shape[0], L), np.int32)
        dist = np.zeros((q.shape[0], L), np.float32)
        check(self.lib.smx_partition_topl(self.h, q.ctypes.data, q.shape[0], L, leaf.ctypes.data,
                                          dist.ctypes.data), "smx_partition_topl")
        return leaf, dist

    def create_lookup_tables(self, queries):
        q = _c(queries, np.float32)
        nb = self.index.num_blocks
        lut = np.zeros((q.shape[0], nb, 16), np.uint8)
        mult = np.zeros(q.shape[0], np.float32)
        check(self.lib.smx_create_lookup_tables(self.h, q.ctypes.data, q.shape[0], lut.ctypes.data,
                                                mult.ctypes.data), "smx_create_lookup_tables")
        return lut, mult

    def exact_distances(self, queries, ids):
        q = _c(queries, np.float32)
        ids = _c(ids, np.uint32)
        out = np.zeros(ids.shape, np.float32)
        check(self.lib.smx_exact_distances(self.h, q.ctypes.data, q.shape[0], ids.ctypes.data,
                                           ids.shape[1], out.ctypes.data), "smx_exact_distances")
        return out

    def leaf_scores(self, leaf, lut_u8):
        lut_u8 = _c(lut_u8, np.uint8)
        n = int(self.index.leaf_offsets[leaf + 1] - self.index.leaf_offsets[leaf])
        out = np.zeros(max(n, 1), np.int32)
        check(self.lib.smx_lut16_leaf_scores(self.h, int(leaf), lut_u8.ctypes.data, out.ctypes.data),
              "smx_lut16_leaf_scores")
        return out[:n]

    def set_profiling(self, on):
        """False / True (mode 1: synchronous per-call stage timings) or 2
        (scan-launch durations of the calls in flight, no synchronisation)."""
        mode = 2 if on == 2 else int(bool(on))
        check(self.lib.smx_set_profiling(self.h, mode), "smx_set_profiling")

    def timings(self):
        t = Timings()
        check(self.lib.smx_get_timings(self.h, ctypes.byref(t)), "smx_get_timings")
        return t.as_dict()

    def set_tuning(self, candidates_per_query: int = 0, seed_leaves: int = 4,
                   scan_variant: int = 0, chunk_tiles: int = 0):
        check(self.lib.smx_set_tuning(self.h, int(candidates_per_query), int(seed_leaves),
                                      int(scan_variant), int(chunk_tiles)), "smx_set_tuning")
