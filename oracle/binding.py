"""ctypes binding of liboracle.so (the CPU restatement).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg.  Never imported by the scann_amd package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

MODE_IDEAL = 0
MODE_EMULATE = 1
PARTITION_ONE_TO_MANY = 4   # or-ed into mode: the single-query partition scores

_f32p = ctypes.POINTER(ctypes.c_float)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_i32p = ctypes.POINTER(ctypes.c_int32)
_u8p = ctypes.POINTER(ctypes.c_uint8)


def build(force: bool = False) -> str:
    """Compile the oracle with its Makefile (gcc)."""
    if force or not os.path.exists(_LIB_PATH):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp = ctypes.c_void_p
        L.orc_partition_scores.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, vp, ctypes.c_int32, ctypes.c_int32, vp]
        L.orc_partition_topl.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp, vp]
        L.orc_create_lut.argtypes = [vp, ctypes.c_int32, vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp, vp, vp]
        L.orc_create_lut.restype = ctypes.c_int
        L.orc_pack_codes.argtypes = [vp, ctypes.c_uint32, ctypes.c_int32, vp]
        L.orc_lut16_accumulate.argtypes = [vp, ctypes.c_uint32, ctypes.c_int32, vp, vp]
        L.orc_global_topn_shift.argtypes = [vp]
        L.orc_global_topn_shift.restype = ctypes.c_int32
        L.orc_search.argtypes = [vp, vp] + [ctypes.c_int32] * 7 + [vp, vp, vp]
        L.orc_search.restype = ctypes.c_int
        L.orc_search_pre_reorder.argtypes = [vp, vp] + [ctypes.c_int32] * 5 + [vp, vp, vp]
        L.orc_search_pre_reorder.restype = ctypes.c_int
        L.orc_exact_distance.argtypes = [vp, vp, ctypes.c_int32, ctypes.c_int32]
        L.orc_exact_distance.restype = ctypes.c_float
        L.orc_fast_topn_replay.argtypes = [vp, vp, ctypes.c_int32, ctypes.c_int32, vp, vp, vp]
        L.orc_fast_topn_replay.restype = ctypes.c_int32
        L.orc_fast_topn_replay_i16.argtypes = [vp, vp, ctypes.c_int32, ctypes.c_int32,
                                               ctypes.c_int16, vp, vp, vp]
        L.orc_fast_topn_replay_i16.restype = ctypes.c_int32
        L.orc_avq_encode.argtypes = [vp, vp, ctypes.c_int32, ctypes.c_int32, vp, ctypes.c_int32,
                                     ctypes.c_int32, ctypes.c_double, vp]
        L.orc_avq_encode.restype = None
        L.orc_avx2_prepare.argtypes = [vp]
        L.orc_avx2_prepare.restype = vp
        L.orc_avx2_release.argtypes = [vp]
        L.orc_search_avx2.argtypes = [vp, vp] + [ctypes.c_int32] * 6 + [vp, vp, vp, vp,
                                                                         ctypes.c_int32]
        L.orc_search_avx2.restype = ctypes.c_int
        _lib = L
    return _lib


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def partition_scores(q, centers, metric):
    q, centers = _c(q, np.float32), _c(centers, np.float32)
    out = np.empty((q.shape[0], centers.shape[0]), np.float32)
    lib().orc_partition_scores(q.ctypes.data, q.shape[0], q.shape[1], centers.ctypes.data,
                               centers.shape[0], metric, out.ctypes.data)
    return out


def partition_topl(q, centers, metric, L):
    q, centers = _c(q, np.float32), _c(centers, np.float32)
    leaf = np.full((q.shape[0], L), -1, np.int32)
    score = np.full((q.shape[0], L), np.nan, np.float32)
    lib().orc_partition_topl(q.ctypes.data, q.shape[0], q.shape[1], centers.ctypes.data,
                             centers.shape[0], metric, L, leaf.ctypes.data, score.ctypes.data)
    return leaf, score


def create_lut(q, codebook, metric):
    q, codebook = _c(q, np.float32), _c(codebook, np.float32)
    nb, _, dpb = codebook.shape
    raw = np.empty(nb * 16, np.float32)
    u8 = np.empty(nb * 16, np.uint8)
    mult = np.zeros(1, np.float32)
    rc = lib().orc_create_lut(q.ctypes.data, q.shape[0], codebook.ctypes.data, nb, dpb, metric,
                              raw.ctypes.data, u8.ctypes.data, mult.ctypes.data)
    if rc != 0:
        raise ValueError("unsupported block layout")
    return raw.reshape(nb, 16), u8.reshape(nb, 16), float(mult[0])


def pack_codes(codes):
    codes = _c(codes, np.uint8)
    n, nb = codes.shape
    out = np.zeros(nb * ((n + 31) // 32) * 16, np.uint8)
    lib().orc_pack_codes(codes.ctypes.data, n, nb, out.ctypes.data)
    return out


def lut16_accumulate(packed, n, nb, lut_u8):
    packed, lut_u8 = _c(packed, np.uint8), _c(lut_u8, np.uint8)
    out = np.empty(n, np.int32)
    lib().orc_lut16_accumulate(packed.ctypes.data, n, nb, lut_u8.ctypes.data, out.ctypes.data)
    return out


def global_topn_shift(index):
    d = index.desc()
    return lib().orc_global_topn_shift(ctypes.byref(d))


def search(index, queries, leaves, pre_nn, final_nn, reorder=True, mode=MODE_IDEAL, nthreads=8):
    q = _c(queries, np.float32)
    nq = q.shape[0]
    d = index.desc()
    idx = np.zeros((nq, final_nn), np.uint32)
    dist = np.zeros((nq, final_nn), np.float32)
    cnt = np.zeros(nq, np.int32)
    rc = lib().orc_search(ctypes.byref(d), q.ctypes.data, nq, leaves, pre_nn, final_nn,
                          int(reorder), mode, nthreads, idx.ctypes.data, dist.ctypes.data,
                          cnt.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"orc_search failed ({rc})")
    return idx, dist, cnt


def search_pre_reorder(index, queries, leaves, pre_nn, mode=MODE_IDEAL, nthreads=8):
    """k' best (global id, AH distance) per query, sorted by (dist, tie id)."""
    q = _c(queries, np.float32)
    nq = q.shape[0]
    width = pre_nn
    d = index.desc()
    idx = np.zeros((nq, width), np.uint32)
    dist = np.zeros((nq, width), np.float32)
    cnt = np.zeros(nq, np.int32)
    rc = lib().orc_search_pre_reorder(ctypes.byref(d), q.ctypes.data, nq, leaves, pre_nn, mode,
                                      nthreads, idx.ctypes.data, dist.ctypes.data, cnt.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"orc_search_pre_reorder failed ({rc})")
    return idx, dist, cnt


def exact_distance(q, x, metric):
    q, x = _c(q, np.float32), _c(x, np.float32)
    return float(lib().orc_exact_distance(q.ctypes.data, x.ctypes.data, q.shape[0], metric))


def fast_topn_replay(ids, dists, k):
    ids, dists = _c(ids, np.uint32), _c(dists, np.float32)
    oi = np.zeros(max(k, 1), np.uint32)
    od = np.zeros(max(k, 1), np.float32)
    ngc = np.zeros(1, np.int32)
    n = lib().orc_fast_topn_replay(ids.ctypes.data, dists.ctypes.data, len(ids), k,
                                   oi.ctypes.data, od.ctypes.data, ngc.ctypes.data)
    return oi[:n], od[:n], int(ngc[0])


def fast_topn_replay_i16(ids, dists, k, epsilon=32767):
    """FastTopNeighbors<int16_t>(k, epsilon) replay; FinishUnsorted storage order."""
    ids, dists = _c(ids, np.uint32), _c(dists, np.int16)
    oi = np.zeros(max(k, 1), np.uint32)
    od = np.zeros(max(k, 1), np.int16)
    ngc = np.zeros(1, np.int32)
    n = lib().orc_fast_topn_replay_i16(ids.ctypes.data, dists.ctypes.data, len(ids), k,
                                       int(epsilon), oi.ctypes.data, od.ctypes.data,
                                       ngc.ctypes.data)
    return oi[:n], od[:n], int(ngc[0])


def avq_encode(residuals, originals, codebook, threshold):
    """The oracle's row-by-row AVQ noise-shaped encoding, uint8 [n, B]."""
    r = _c(residuals, np.float32)
    x = _c(originals, np.float32)
    cb = _c(codebook, np.float32)
    nb, _, dpb = cb.shape
    out = np.zeros((r.shape[0], nb), np.uint8)
    lib().orc_avq_encode(r.ctypes.data, x.ctypes.data, r.shape[0], r.shape[1], cb.ctypes.data,
                         nb, dpb, float(threshold), out.ctypes.data)
    return out


class Avx2Port:
    """The AVX2 port (cpu_baseline).  Keeps the index alive while prepared."""

    def __init__(self, index):
        self.index = index
        self._desc = index.desc()
        self._h = lib().orc_avx2_prepare(ctypes.byref(self._desc))
        if not self._h:
            raise ValueError("index not covered by the AVX2 port (residual indexes need the global top-N path)")

    def search(self, queries, leaves, pre_nn, final_nn, reorder=True, nthreads=8,
               batch_shared=True):
        q = _c(queries, np.float32)
        nq = q.shape[0]
        idx = np.zeros((nq, final_nn), np.uint32)
        dist = np.zeros((nq, final_nn), np.float32)
        cnt = np.zeros(nq, np.int32)
        ph = np.zeros(3, np.float64)
        rc = lib().orc_search_avx2(self._h, q.ctypes.data, nq, leaves, pre_nn, final_nn,
                                   int(reorder), nthreads, idx.ctypes.data, dist.ctypes.data,
                                   cnt.ctypes.data, ph.ctypes.data, int(bool(batch_shared)))
        if rc != 0:
            raise RuntimeError(f"orc_search_avx2 failed ({rc})")
        # CPU seconds (summed over threads) of the last call: partition +
        # top-L + LUT, the leaf scan (LUT16 + FastTopNeighbors), finish +
        # dedupe + reorder
        self.last_phase_s = dict(front=float(ph[0]), scan=float(ph[1]), tail=float(ph[2]))
        return idx, dist, cnt

    def close(self):
        if self._h:
            lib().orc_avx2_release(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
