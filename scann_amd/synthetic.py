"""Seeded synthetic stand-ins for the BASELINE.json datasets (no network).

glove-100-angular is replaced by a unit-normalised Gaussian mixture of the
same shape; SIFT1M by non-negative rounded mixture
vectors (config 3).  Queries are fresh draws from the same mixture.
"""
from __future__ import annotations

import numpy as np

GLOVE_N, GLOVE_D = 1_183_514, 100
SIFT_N, SIFT_D = 1_000_000, 128
# SIFT1M stand-in: 100 broad components (noise norm 0.8 against unit means,
# then |x| * 256 rounded to bytes), so that a query's neighbourhood spans
# several of the 2000 leaves and recall rises with leaves_to_search
# (partition recall of the true top-10 at L = 10 / 20 / 50: 0.83 / 0.99 /
# 0.998, against 1.0 already at L = 10 with round 4's 1000 tight
# components, which made the recall sweep flat)
SIFT_COMPONENTS, SIFT_SPREAD = 100, 0.8


def mixture(n: int, d: int, components: int, spread: float, seed: int,
            normalize: bool = True, chunk: int = 1 << 18,
            means_seed: int | None = None) -> np.ndarray:
    """Rows = unit mean + N(0, spread^2/d); optionally L2-normalised."""
    mrng = np.random.default_rng(seed if means_seed is None else means_seed)
    means = mrng.standard_normal((components, d)).astype(np.float32)
    means /= np.linalg.norm(means, axis=1, keepdims=True)
    rng = np.random.default_rng(seed + 1)
    out = np.empty((n, d), np.float32)
    sigma = np.float32(spread / np.sqrt(d))
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        z = rng.integers(0, components, m)
        x = means[z] + sigma * rng.standard_normal((m, d), dtype=np.float32)
        if normalize:
            x /= np.linalg.norm(x, axis=1, keepdims=True)
        out[s:s + m] = x
    return out


def glove_like(n: int = GLOVE_N, nq: int = 1000, d: int = GLOVE_D, seed: int = 2,
               components: int = 2000, spread: float = 0.9):
    db = mixture(n, d, components, spread, seed, means_seed=seed)
    q = mixture(nq, d, components, spread, seed + 100, means_seed=seed)
    return db, q


def sift_draw(m: int, s: int, seed: int = 3, d: int = SIFT_D,
              components: int = SIFT_COMPONENTS, spread: float = SIFT_SPREAD) -> np.ndarray:
    """m SIFT-like rows (non-negative, rounded to bytes) drawn with seed `s`
    from the mixture whose means come from `seed`."""
    x = mixture(m, d, components, spread, s, normalize=False, means_seed=seed)
    return np.clip(np.rint(np.abs(x) * 256.0), 0, 255).astype(np.float32)


def sift_like(n: int = SIFT_N, nq: int = 1000, d: int = SIFT_D, seed: int = 3,
              components: int = SIFT_COMPONENTS, spread: float = SIFT_SPREAD):
    return (sift_draw(n, seed, seed, d, components, spread),
            sift_draw(nq, seed + 100, seed, d, components, spread))


def brute_force_topk(db: np.ndarray, q: np.ndarray, k: int, metric: int,
                     chunk: int = 1 << 17) -> np.ndarray:
    """Exact top-k ids (float64 scores); torch GPU when available."""
    try:
        import torch
        use_t = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        use_t = False
    nq = q.shape[0]
    best_s = np.full((nq, k), np.inf)
    best_i = np.zeros((nq, k), np.int64)
    if use_t:
        dev = torch.device("cuda")
        qt = torch.from_numpy(q).to(dev, torch.float64)
        qn = (qt * qt).sum(1, keepdim=True)
    for s in range(0, db.shape[0], chunk):
        if use_t:
            xb = torch.from_numpy(db[s:s + chunk]).to(dev, torch.float64)
            ip = qt @ xb.T
            sc = -ip if metric == 0 else qn - 2 * ip + (xb * xb).sum(1)[None, :]
            kk = min(k, sc.shape[1])
            v, i = torch.topk(sc, kk, dim=1, largest=False)
            v, i = v.cpu().numpy(), i.cpu().numpy() + s
        else:
            xb = db[s:s + chunk].astype(np.float64)
            ip = q.astype(np.float64) @ xb.T
            sc = -ip if metric == 0 else (q.astype(np.float64) ** 2).sum(1)[:, None] - 2 * ip + (xb ** 2).sum(1)[None, :]
            kk = min(k, sc.shape[1])
            i = np.argpartition(sc, kk - 1, axis=1)[:, :kk]
            v = np.take_along_axis(sc, i, 1)
            i = i + s
        allv = np.concatenate([best_s, v], 1)
        alli = np.concatenate([best_i, i], 1)
        o = np.argsort(allv, axis=1, kind="stable")[:, :k]
        best_s = np.take_along_axis(allv, o, 1)
        best_i = np.take_along_axis(alli, o, 1)
    return best_i


def recall_at_k(found: np.ndarray, truth: np.ndarray, k: int) -> float:
    hits = 0
    for f, t in zip(found[:, :k], truth[:, :k]):
        hits += len(set(f.tolist()) & set(t.tolist()))
    return hits / float(truth.shape[0] * k)
