"""Index construction on the GPU: every step in the hand-written HIP kernels of
scann_amd/csrc/smx_builder.hip and smx_sort.hip (torch holds the device
buffers and picks random rows; it computes nothing).

* k-means partitioner (GmmUtils::KMeansImpl, gmm_utils.cc:539-1318): random
  initial centers from a sample, Lloyd steps with the assignment in
  smx_nearest_centers and the mean step as exact fixed-point sums
  (smx_kmeans_accumulate / smx_kmeans_finalize: order-independent, so the
  centers are the same run to run), empty centers re-seeded from the sample;
* tokenization: nearest center of every row, and with SOAR the spilled
  center (kmeans_tree_partitioner.cc:926-997), both smx_nearest_centers;
* datapoints_by_token: members grouped by (leaf, id) on the device
  (smx_group_by_leaf: a radix sort of leaf << 32 | id);
* residuals x - c_leaf (smx_gather_residuals);
* the AH codebook: 16-center k-means per block on a residual sample
  (asymmetric_hashing_impl.cc:41-198; smx_block_encode assigns every block
  at once, smx_codebook_accumulate sums every block at once);
* codes: nearest codebook center per block (smx_block_encode) or the
  anisotropic noise-shaped codes (smx_avq_encode, IndexDatapointNoiseShaped,
  asymmetric_hashing_impl.cc:434-503; bit for bit the oracle's
  orc_avq_encode).

The result is the same TreeAHIndex the host builder produces (the trainer's
random choices differ, so the indexes differ in training noise only; no
parity claim depends on the build, whose output is the input of both the GPU
search and the oracle).
"""
from __future__ import annotations

import ctypes
import math
import time
from typing import Optional

import numpy as np

from . import _native
from .index import METRIC_DOT, TreeAHIndex


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("device_builder needs a GPU (the build kernels are HIP)")
    return torch


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def _stream():
    return _native._current_stream(None)


def fixed_point_scale(max_abs: float, n: int) -> float:
    """A power of two s with n * max_abs * s < 2^62: no fixed-point sum of n
    values of magnitude <= max_abs overflows int64."""
    m = max(float(max_abs), 1e-30) * max(1, int(n))
    return float(2.0 ** (61 - math.ceil(math.log2(m))))


def nearest_centers(x, centers, primary=None, lam: float = 0.0, out=None):
    torch = _torch()
    n, d = x.shape
    out = out if out is not None else torch.empty(n, dtype=torch.int32, device=x.device)
    _native.nearest_centers_device(_p(x), n, d, _p(centers), centers.shape[0], _p(out),
                                   None if primary is None else _p(primary), float(lam))
    return out


def kmeans(x, k: int, iterations: int, seed: int, rng=None):
    """Lloyd's k-means of the device rows x [n, d] (float32) into k centers."""
    torch = _torch()
    rng = rng or np.random.default_rng(seed)
    n, d = x.shape
    dev = x.device
    if k >= n:
        c = torch.zeros((k, d), dtype=torch.float32, device=dev)
        c[:n] = x
        return c
    idx = torch.from_numpy(rng.choice(n, k, replace=False).astype(np.int64)).to(dev)
    centers = x[idx].contiguous()
    labels = torch.empty(n, dtype=torch.int32, device=dev)
    sums = torch.empty(k * d, dtype=torch.int64, device=dev)
    counts = torch.empty(k, dtype=torch.int32, device=dev)
    scale = fixed_point_scale(float(x.abs().max()), n)
    lib = _native.load()
    for _ in range(iterations):
        nearest_centers(x, centers, out=labels)
        sums.zero_()
        counts.zero_()
        _native.check(lib.smx_kmeans_accumulate(_p(x), n, d, _p(labels), k, scale, _p(sums),
                                                _p(counts), _stream()), "smx_kmeans_accumulate")
        _native.check(lib.smx_kmeans_finalize(_p(sums), _p(counts), k, d, scale, _p(centers),
                                              _stream()), "smx_kmeans_finalize")
        empty = np.flatnonzero(counts.cpu().numpy() == 0)
        if empty.size:
            pick = torch.from_numpy(rng.choice(n, empty.size, replace=False).astype(np.int64))
            centers[torch.from_numpy(empty).to(dev)] = x[pick.to(dev)]
    return centers


def block_encode(rows, codebook, out=None):
    torch = _torch()
    n, dim = rows.shape
    nb, _, dpb = codebook.shape
    out = out if out is not None else torch.empty((n, nb), dtype=torch.uint8, device=rows.device)
    _native.check(_native.load().smx_block_encode(_p(rows), n, dim, _p(codebook), nb, dpb,
                                                  _p(out), _stream()), "smx_block_encode")
    return out


def avq_encode(residuals, datapoints, codebook, threshold: float, out=None):
    torch = _torch()
    n, dim = residuals.shape
    nb, _, dpb = codebook.shape
    out = out if out is not None else torch.empty((n, nb), dtype=torch.uint8,
                                                  device=residuals.device)
    _native.check(_native.load().smx_avq_encode(_p(residuals), _p(datapoints), n, dim,
                                                _p(codebook), nb, dpb, float(threshold), _p(out),
                                                _stream()), "smx_avq_encode")
    return out


def train_codebook(residuals, num_blocks: int, dpb: int, iterations: int, seed: int):
    """16-center k-means per block of the device rows [n, dim]; every block's
    assignment and mean step in one launch each.  Per block, the initial
    centers and re-seeds come from its own generator (seed + 7919 b), as in
    index_builder.train_codebook."""
    torch = _torch()
    n, dim = residuals.shape
    dev = residuals.device
    pad = num_blocks * dpb - dim
    padded = residuals if pad == 0 else torch.cat(
        [residuals, torch.zeros((n, pad), dtype=torch.float32, device=dev)], 1)
    blocks = padded.view(n, num_blocks, dpb)
    rngs = [np.random.default_rng(seed + 7919 * b) for b in range(num_blocks)]
    cb = torch.zeros((num_blocks, 16, dpb), dtype=torch.float32, device=dev)
    if n <= 16:
        cb[:, :n] = blocks.permute(1, 0, 2)
        return cb
    for b in range(num_blocks):
        idx = torch.from_numpy(rngs[b].choice(n, 16, replace=False).astype(np.int64)).to(dev)
        cb[b] = blocks[idx, b]
    codes = torch.empty((n, num_blocks), dtype=torch.uint8, device=dev)
    sums = torch.empty(num_blocks * 16 * dpb, dtype=torch.int64, device=dev)
    counts = torch.empty(num_blocks * 16, dtype=torch.int32, device=dev)
    scale = fixed_point_scale(float(residuals.abs().max()), n)
    lib = _native.load()
    for _ in range(iterations):
        block_encode(residuals, cb, out=codes)
        sums.zero_()
        counts.zero_()
        _native.check(lib.smx_codebook_accumulate(_p(residuals), n, dim, _p(codes), num_blocks,
                                                  dpb, scale, _p(sums), _p(counts), _stream()),
                      "smx_codebook_accumulate")
        _native.check(lib.smx_kmeans_finalize(_p(sums), _p(counts), num_blocks * 16, dpb, scale,
                                              _p(cb), _stream()), "smx_kmeans_finalize")
        cnt = counts.cpu().numpy().reshape(num_blocks, 16)
        for b in np.flatnonzero((cnt == 0).any(1)):
            empty = np.flatnonzero(cnt[b] == 0)
            pick = torch.from_numpy(rngs[b].choice(n, empty.size, replace=False).astype(np.int64))
            cb[b, torch.from_numpy(empty).to(dev)] = blocks[pick.to(dev), b]
    return cb


def group_by_leaf(labels, ids, k: int):
    """(offsets [k + 1] uint64, members [m] uint32 as int32 storage, member
    leaf [m] int32) of the (label, id) pairs, members of a leaf by ascending
    id."""
    torch = _torch()
    m = labels.numel()
    dev = labels.device
    lib = _native.load()
    tb = ctypes.c_size_t(0)
    _native.check(lib.smx_group_by_leaf(None, None, m, k, None, ctypes.byref(tb), None, None,
                                        None, None, _stream()), "smx_group_by_leaf")
    temp = torch.empty(max(1, tb.value), dtype=torch.uint8, device=dev)
    keys = torch.empty(max(1, 2 * m), dtype=torch.int64, device=dev)
    offsets = torch.empty(k + 1, dtype=torch.int64, device=dev)
    members = torch.empty(max(1, m), dtype=torch.int32, device=dev)
    member_leaf = torch.empty(max(1, m), dtype=torch.int32, device=dev)
    _native.check(lib.smx_group_by_leaf(_p(labels), _p(ids), m, k, _p(temp), ctypes.byref(tb),
                                        _p(keys), _p(offsets), _p(members), _p(member_leaf),
                                        _stream()), "smx_group_by_leaf")
    return offsets, members[:m], member_leaf[:m]


def gather_residuals(x, rows, leaf, centers, row_base: int = 0, out=None):
    """out[i] = x[rows[i] - row_base] - centers[leaf[i]] (centers None: the row)."""
    torch = _torch()
    m = rows.numel()
    d = x.shape[1]
    out = out if out is not None else torch.empty((m, d), dtype=torch.float32, device=x.device)
    _native.check(_native.load().smx_gather_residuals(
        _p(x), d, _p(rows), None if leaf is None else _p(leaf),
        None if centers is None else _p(centers), m, int(row_base), _p(out), _stream()),
        "smx_gather_residuals")
    return out


def build_tree_ah(db, metric: int, num_leaves: int, dims_per_block: int = 2, *,
                  training_sample_size: int = 100000, training_iterations: int = 12,
                  ah_training_iterations: int = 10, ah_training_sample_size: int = 100000,
                  residual: Optional[bool] = None, keep_dataset: bool = True,
                  soar_lambda: Optional[float] = None, overretrieve_factor: float = 2.0,
                  seed: int = 0, noise_shaping_threshold: Optional[float] = None,
                  timings: Optional[dict] = None) -> TreeAHIndex:
    """index_builder.build_tree_ah's index, every step on the GPU.  `db` is a
    host array or a device tensor [n, dim] float32; `timings` (a dict)
    receives the seconds of each phase (device-synchronised)."""
    torch = _torch()
    t_all = time.perf_counter()
    marks = {}

    def mark(name, t0):
        torch.cuda.synchronize()
        marks[name] = time.perf_counter() - t0
        return time.perf_counter()

    t = time.perf_counter()
    x = db if isinstance(db, torch.Tensor) else torch.from_numpy(
        np.ascontiguousarray(db, dtype=np.float32))
    x = x.to(device="cuda", dtype=torch.float32).contiguous()
    n, dim = x.shape
    dev = x.device
    if residual is None:
        residual = metric == METRIC_DOT
    num_leaves = max(1, min(num_leaves, n))
    t = mark("upload", t)
    rng = np.random.default_rng(seed)
    samp = x
    if n > training_sample_size:
        sel = np.sort(rng.choice(n, training_sample_size, replace=False)).astype(np.int64)
        samp = x[torch.from_numpy(sel).to(dev)]
    centers = kmeans(samp, num_leaves, training_iterations, seed, rng=rng)
    del samp
    t = mark("partitioner", t)
    labels = nearest_centers(x, centers)
    ids = torch.arange(n, dtype=torch.int32, device=dev)
    if soar_lambda is not None and num_leaves > 1:
        second = nearest_centers(x, centers, primary=labels, lam=float(soar_lambda))
        labels = torch.cat([labels, second])
        ids = torch.cat([ids, ids])
    t = mark("tokenize", t)
    offsets, members, member_leaf = group_by_leaf(labels, ids, num_leaves)
    del labels, ids
    t = mark("group", t)
    resid = gather_residuals(x, members, member_leaf, centers if residual else None)
    m = members.numel()
    num_blocks = int(math.ceil(dim / dims_per_block))
    rng2 = np.random.default_rng(seed + 1)
    asamp = resid
    if m > ah_training_sample_size:
        sel = np.sort(rng2.choice(m, ah_training_sample_size, replace=False)).astype(np.int64)
        asamp = resid[torch.from_numpy(sel).to(dev)]
    codebook = train_codebook(asamp, num_blocks, dims_per_block, ah_training_iterations, seed + 2)
    del asamp
    t = mark("codebook", t)
    if noise_shaping_threshold is not None and not math.isnan(noise_shaping_threshold):
        # AVQ: the parallel direction is the datapoint's own row
        orig = gather_residuals(x, members, None, None)
        codes = avq_encode(resid, orig, codebook, float(noise_shaping_threshold))
        del orig
    else:
        codes = block_encode(resid, codebook)
    del resid
    t = mark("encode", t)
    out = TreeAHIndex(metric=metric, dim=dim, num_blocks=num_blocks,
                      dims_per_block=dims_per_block, residual=bool(residual),
                      centers=centers.cpu().numpy(), codebook=codebook.cpu().numpy(),
                      leaf_offsets=offsets.cpu().numpy().astype(np.uint64),
                      leaf_members=members.cpu().numpy().view(np.uint32),
                      member_codes=codes.cpu().numpy(), num_datapoints=n,
                      dataset=(x.cpu().numpy() if not isinstance(db, np.ndarray) else
                               np.ascontiguousarray(db, dtype=np.float32))
                      if keep_dataset else None,
                      spilling_overretrieve_factor=float(overretrieve_factor))
    mark("download", t)
    marks["total"] = time.perf_counter() - t_all
    if timings is not None:
        timings.update(marks)
    return out
