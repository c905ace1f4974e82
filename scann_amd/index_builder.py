"""Index construction for the tree-AH (LUT16) searcher.

Build time is outside the hot path of this tier (SURVEY.md §8f-3 ranks the
GPU index builder as a "next" row).  This module trains what the query path
needs so that the searcher can be used end to end from the reference's
builder API:

* the k-means partitioner (squared-L2 partitioning distance, random
  initialisation, ``training_iterations`` rounds on a ``training_sample_size``
  sample; reference: scann/utils/gmm_utils.cc, kmeans_tree_partitioner.cc);
* database tokenization by squared-L2 top-1 with ``datapoints_by_token``
  sorted by global id (kmeans_tree_partitioner.cc:477-620, 532-535);
* residuals against the assigned center for tree + dot product
  (tree_ah_hybrid_residual.cc:185-224, scann_builder.py:429-431);
* one 16-center k-means codebook per block (asymmetric_hashing_impl.cc:41-198)
  and nearest-center encoding, or -- with a noise_shaping_threshold (the
  builder's anisotropic_quantization_threshold) -- the anisotropic (AVQ)
  noise-shaped encoding of IndexDatapointNoiseShaped
  (asymmetric_hashing_impl.cc:268-503), on the GPU when one is visible;
* optional SOAR spilling: a second leaf per datapoint minimising
  ||x - c||^2 + lambda * <r, x - c>^2 / ||r||^2 with r the primary residual
  (SOAR's orthogonality-amplified loss, kmeans_tree_partitioner.cc:926-997),
  encoded against that leaf's center.

On a GPU the row-to-center assignments (k-means steps, partitioning, SOAR)
run in the hand-written HIP kernel smx_nearest_centers
(scann_amd/csrc/smx_builder.hip) and the AVQ encoder and codebook encoding
in torch; numpy otherwise.  Results differ only in training floating-point
noise, which no parity claim depends on (the built index is the input of
both the GPU path and the oracle).
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np

from .index import METRIC_DOT, TreeAHIndex


def _torch_device():
    try:
        import torch
        if torch.cuda.is_available():
            return torch, torch.device("cuda")
    except Exception:  # pragma: no cover - torch is optional for building
        pass
    return None, None


def _hip_nearest(x: np.ndarray, centers: np.ndarray, primary: Optional[np.ndarray] = None,
                 lam: float = 0.0, chunk: int = 1 << 20) -> np.ndarray:
    """The hand-written HIP assignment kernel (smx_nearest_centers,
    scann_amd/csrc/smx_builder.hip) on rows streamed to the device in chunks."""
    import torch
    from . import _native
    dev = torch.device("cuda")
    c = torch.from_numpy(np.ascontiguousarray(centers, dtype=np.float32)).to(dev)
    k, d = c.shape
    out = np.empty(x.shape[0], dtype=np.int64)
    res = torch.empty(min(chunk, max(1, x.shape[0])), dtype=torch.int32, device=dev)
    for s in range(0, x.shape[0], chunk):
        xb = torch.from_numpy(np.ascontiguousarray(x[s:s + chunk], dtype=np.float32)).to(dev)
        m = xb.shape[0]
        pb = None
        if primary is not None:
            pb = torch.from_numpy(np.ascontiguousarray(primary[s:s + chunk], dtype=np.int32)).to(dev)
        _native.nearest_centers_device(xb.data_ptr(), m, d, c.data_ptr(), k, res.data_ptr(),
                                       None if pb is None else pb.data_ptr(), lam)
        out[s:s + m] = res[:m].cpu().numpy()
    return out


def _assign_l2(x: np.ndarray, centers: np.ndarray, chunk: int = 1 << 16) -> np.ndarray:
    """argmin_c ||x - c||^2 for every row of x (ties -> lowest index): the
    HIP kernel when a GPU is visible, numpy otherwise."""
    torch, dev = _torch_device()
    if torch is not None:
        return _hip_nearest(x, centers)
    out = np.empty(x.shape[0], dtype=np.int64)
    # bound one distance block to ~2^28 entries (50000 centers: 5k rows)
    chunk = max(1024, min(chunk, (1 << 28) // max(1, centers.shape[0])))
    cn = (centers * centers).sum(1)
    for s in range(0, x.shape[0], chunk):
        d = cn[None, :] - 2.0 * (x[s:s + chunk] @ centers.T)
        out[s:s + chunk] = d.argmin(1)
    return out


def kmeans(x: np.ndarray, k: int, iterations: int, seed: int,
           sample_size: Optional[int] = None) -> np.ndarray:
    """Lloyd's k-means with random initialisation; empty clusters re-seeded."""
    rng = np.random.default_rng(seed)
    n = x.shape[0]
    if sample_size is not None and n > sample_size:
        x = x[np.sort(rng.choice(n, sample_size, replace=False))]
        n = sample_size
    if k >= n:
        c = np.zeros((k, x.shape[1]), np.float32)
        c[:n] = x
        return c
    centers = x[rng.choice(n, k, replace=False)].astype(np.float32, copy=True)
    for _ in range(iterations):
        lab = _assign_l2(x, centers)
        cnt = np.bincount(lab, minlength=k)
        # per-center sums: sort by label, reduce each run (np.add.at is slow)
        order = np.argsort(lab, kind="stable")
        starts = np.concatenate([[0], np.cumsum(cnt)[:-1]])
        nzs = cnt > 0
        sums = np.zeros_like(centers, dtype=np.float64)
        if nzs.any():
            sums[nzs] = np.add.reduceat(x[order].astype(np.float64), starts[nzs], axis=0)
        nz = cnt > 0
        centers[nz] = (sums[nz] / cnt[nz, None]).astype(np.float32)
        if (~nz).any():
            centers[~nz] = x[rng.choice(n, int((~nz).sum()), replace=False)]
    return centers


def _block_view(v: np.ndarray, num_blocks: int, dpb: int) -> np.ndarray:
    """[n, D] -> [n, B, dpb] with the last block zero-padded."""
    n, d = v.shape
    pad = num_blocks * dpb - d
    if pad:
        v = np.concatenate([v, np.zeros((n, pad), v.dtype)], axis=1)
    return v.reshape(n, num_blocks, dpb)


def train_codebook(residuals: np.ndarray, num_blocks: int, dpb: int,
                   iterations: int, seed: int) -> np.ndarray:
    blocks = _block_view(residuals, num_blocks, dpb)
    cb = np.zeros((num_blocks, 16, dpb), np.float32)
    for b in range(num_blocks):
        cb[b] = kmeans(np.ascontiguousarray(blocks[:, b, :]), 16, iterations, seed + 7919 * b)
    return cb


def encode(residuals: np.ndarray, codebook: np.ndarray, chunk: int = 1 << 15) -> np.ndarray:
    """Nearest codebook center per block (squared L2), uint8 [n, B]."""
    num_blocks, _, dpb = codebook.shape
    n = residuals.shape[0]
    out = np.empty((n, num_blocks), np.uint8)
    torch, dev = _torch_device()
    if torch is not None:
        cb = torch.from_numpy(codebook).to(dev)
        for s in range(0, n, chunk):
            r = torch.from_numpy(_block_view(residuals[s:s + chunk], num_blocks, dpb)).to(dev)
            d = ((r[:, :, None, :] - cb[None]) ** 2).sum(-1)
            out[s:s + chunk] = d.argmin(-1).to(torch.uint8).cpu().numpy()
        return out
    for s in range(0, n, chunk):
        r = _block_view(residuals[s:s + chunk], num_blocks, dpb)
        d = ((r[:, :, None, :] - codebook[None]) ** 2).sum(-1)
        out[s:s + chunk] = d.argmin(-1)
    return out


def _avq_parallel_cost_multiplier(t: float, sq_norm, dims: int):
    """ComputeParallelCostMultiplier (asymmetric_hashing_impl.cc:268-274)."""
    parallel = (t * t) / sq_norm
    perpendicular = (1.0 - (t * t) / sq_norm) / (dims - 1.0)
    return parallel / perpendicular


def encode_avq(residuals: np.ndarray, originals: np.ndarray, codebook: np.ndarray,
               threshold: float, chunk: int = 1 << 15) -> np.ndarray:
    """Noise-shaped (AVQ) codes, uint8 [n, B]: IndexDatapointNoiseShaped
    (asymmetric_hashing_impl.cc:434-503) for every row, vectorised over rows.

    Per row, in double: the per-block, per-center residual norm sum (r - c)^2
    and parallel component sum (r - c) * x / ||x|| (ComputeResidualStats,
    :283-343; sums over a block's dims in dim order); start from each block's
    nearest center (InitializeToMinResidualNorm, first minimum); blocks
    visited by their residual norm, largest first; up to 10 rounds of
    coordinate descent where a block moves to the center with the most
    negative eta * d_parallel^2 + d_perpendicular among those that do not
    grow the parallel component (OptimizeSingleSubspace, :366-404, first
    minimum in center order).  A row whose round changes nothing would repeat
    it, so running every row 10 rounds equals the reference's early exit.
    Ties between equal block residual norms keep block order (the
    reference's ZipSortBranchOptimized leaves their order unspecified)."""
    num_blocks, nc, dpb = codebook.shape
    n, dim = originals.shape
    out = np.empty((n, num_blocks), np.uint8)
    torch, dev = _torch_device()
    if torch is not None:
        xp_from = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    else:
        xp_from = lambda a: a  # noqa: E731
    cb = xp_from(codebook.astype(np.float64))                    # [B, 16, dpb]
    for s in range(0, n, chunk):
        r = xp_from(_block_view(residuals[s:s + chunk], num_blocks, dpb).astype(np.float64))
        x = xp_from(_block_view(originals[s:s + chunk], num_blocks, dpb).astype(np.float64))
        m = r.shape[0]
        # ||x||^2 accumulated over the chunked coordinates in order; 1/sqrt
        sqn = None
        for b in range(num_blocks):
            for i in range(dpb):
                t = x[:, b, i] * x[:, b, i]
                sqn = t if sqn is None else sqn + t
        inv_norm = 1.0 / (torch.sqrt(sqn) if torch is not None else np.sqrt(sqn))
        rn = None
        par = None
        for i in range(dpb):
            d = r[:, :, None, i] - cb[None, :, :, i]                  # [m, B, 16]
            t_rn = d * d
            t_par = (d * x[:, :, None, i]) * inv_norm[:, None, None]
            rn = t_rn if rn is None else rn + t_rn
            par = t_par if par is None else par + t_par
        eta = _avq_parallel_cost_multiplier(float(threshold), sqn, dim)     # [m]
        if torch is not None:
            codes = torch.argmin(rn, dim=2)                                  # first minimum
            rows = torch.arange(m, device=dev)
            cur_par = torch.gather(par, 2, codes[:, :, None])[:, :, 0]
            P = torch.zeros(m, dtype=torch.float64, device=dev)
            for b in range(num_blocks):
                P = P + cur_par[:, b]
            cur_rn = torch.gather(rn, 2, codes[:, :, None])[:, :, 0]
            order = torch.argsort(-cur_rn, dim=1, stable=True)
            kidx = torch.arange(nc, device=dev)[None, :]
            inf = torch.tensor(float("inf"), dtype=torch.float64, device=dev)
            for _ in range(10):
                for i in range(num_blocks):
                    b = order[:, i]
                    st_rn = rn[rows, b]                                      # [m, 16]
                    st_par = par[rows, b]
                    cur = codes[rows, b]
                    old_rn = st_rn[rows, cur]
                    old_par = st_par[rows, cur]
                    new_p = (P - old_par)[:, None] + st_par
                    pnd = new_p * new_p - (P * P)[:, None]
                    rnd = st_rn - old_rn[:, None]
                    cost = eta[:, None] * pnd + (rnd - pnd)
                    ok = (pnd <= 0.0) & (kidx != cur[:, None])
                    cost = torch.where(ok, cost, inf)
                    best = torch.argmin(cost, dim=1)
                    take = cost[rows, best] < 0.0
                    codes[rows[take], b[take]] = best[take]
                    P = torch.where(take, new_p[rows, best], P)
            out[s:s + m] = codes.to(torch.uint8).cpu().numpy()
        else:
            codes = np.argmin(rn, axis=2)
            rows = np.arange(m)
            cur_par = np.take_along_axis(par, codes[:, :, None], 2)[:, :, 0]
            P = np.zeros(m)
            for b in range(num_blocks):
                P = P + cur_par[:, b]
            cur_rn = np.take_along_axis(rn, codes[:, :, None], 2)[:, :, 0]
            order = np.argsort(-cur_rn, axis=1, kind="stable")
            kidx = np.arange(nc)[None, :]
            for _ in range(10):
                for i in range(num_blocks):
                    b = order[:, i]
                    st_rn = rn[rows, b]
                    st_par = par[rows, b]
                    cur = codes[rows, b]
                    old_rn = st_rn[rows, cur]
                    old_par = st_par[rows, cur]
                    new_p = (P - old_par)[:, None] + st_par
                    pnd = new_p * new_p - (P * P)[:, None]
                    rnd = st_rn - old_rn[:, None]
                    cost = eta[:, None] * pnd + (rnd - pnd)
                    ok = (pnd <= 0.0) & (kidx != cur[:, None])
                    cost = np.where(ok, cost, np.inf)
                    best = np.argmin(cost, axis=1)
                    take = cost[rows, best] < 0.0
                    codes[rows[take], b[take]] = best[take]
                    P = np.where(take, new_p[rows, best], P)
            out[s:s + m] = codes.astype(np.uint8)
    return out


def soar_assign(x: np.ndarray, centers: np.ndarray, primary: np.ndarray, lam: float,
                chunk: int = 1 << 15) -> np.ndarray:
    """Secondary leaf per row with the SOAR loss (never the primary leaf): the
    HIP kernel when a GPU is visible, numpy otherwise."""
    torch, dev = _torch_device()
    if torch is not None:
        return _hip_nearest(x, centers, primary=primary, lam=float(lam))
    out = np.empty(x.shape[0], dtype=np.int64)
    chunk = max(1024, min(chunk, (1 << 27) // max(1, centers.shape[0])))
    cn = (centers * centers).sum(1)
    for s in range(0, x.shape[0], chunk):
        xb, p = x[s:s + chunk], primary[s:s + chunk]
        r = xb - centers[p]
        rn = np.maximum((r * r).sum(1), 1e-30)
        d2 = (xb * xb).sum(1, keepdims=True) - 2.0 * (xb @ centers.T) + cn[None, :]
        proj = (r * xb).sum(1, keepdims=True) - r @ centers.T
        loss = d2 + lam * proj * proj / rn[:, None]
        loss[np.arange(xb.shape[0]), p] = np.inf
        out[s:s + chunk] = loss.argmin(1)
    return out


def build_tree_ah(db: np.ndarray, metric: int, num_leaves: int,
                  dims_per_block: int = 2, *, training_sample_size: int = 100000,
                  training_iterations: int = 12, ah_training_iterations: int = 10,
                  ah_training_sample_size: int = 100000, residual: Optional[bool] = None,
                  keep_dataset: bool = True, soar_lambda: Optional[float] = None,
                  overretrieve_factor: float = 2.0, seed: int = 0,
                  noise_shaping_threshold: Optional[float] = None) -> TreeAHIndex:
    db = np.ascontiguousarray(db, dtype=np.float32)
    n, dim = db.shape
    if residual is None:
        residual = metric == METRIC_DOT
    num_leaves = max(1, min(num_leaves, n))
    centers = kmeans(db, num_leaves, training_iterations, seed, training_sample_size)
    labels = _assign_l2(db, centers)
    ids = np.arange(n, dtype=np.int64)
    if soar_lambda is not None and num_leaves > 1:
        second = soar_assign(db, centers, labels, float(soar_lambda))
        ids = np.concatenate([ids, ids])
        labels = np.concatenate([labels, second])
    order = np.lexsort((ids, labels))          # by leaf, then ascending id
    counts = np.bincount(labels, minlength=num_leaves)
    offsets = np.zeros(num_leaves + 1, np.uint64)
    offsets[1:] = np.cumsum(counts)
    members = ids[order].astype(np.uint32)
    member_leaf = labels[order]
    num_blocks = int(math.ceil(dim / dims_per_block))
    resid = db[members] - centers[member_leaf] if residual else db[members]
    rng = np.random.default_rng(seed + 1)
    samp = resid
    if resid.shape[0] > ah_training_sample_size:
        samp = resid[np.sort(rng.choice(resid.shape[0], ah_training_sample_size, replace=False))]
    codebook = train_codebook(samp, num_blocks, dims_per_block, ah_training_iterations, seed + 2)
    if noise_shaping_threshold is not None and not math.isnan(noise_shaping_threshold):
        # AVQ: the parallel direction is the datapoint's own (the original
        # row, for a residual index and for a SOAR copy alike)
        codes = encode_avq(resid, db[members], codebook, float(noise_shaping_threshold))
    else:
        codes = encode(resid, codebook)
    return TreeAHIndex(metric=metric, dim=dim, num_blocks=num_blocks,
                       dims_per_block=dims_per_block, residual=bool(residual),
                       centers=centers, codebook=codebook, leaf_offsets=offsets,
                       leaf_members=members, member_codes=codes, num_datapoints=n,
                       dataset=db if keep_dataset else None,
                       spilling_overretrieve_factor=float(overretrieve_factor))
