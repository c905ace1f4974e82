"""The index-build assignment kernel (smx_nearest_centers,
scann_amd/csrc/smx_builder.hip) against float64 restatements of the
reference's losses: the k-means nearest center (gmm_utils.cc:539-1318,
ties to the lowest index) and the SOAR secondary center
(kmeans_tree_partitioner.cc:926-997, primary excluded).  The kernel computes
in f32, so rows whose best two float64 losses are within a relative 1e-4 may
legitimately differ; every other row must match exactly."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(x, c, primary=None, lam=0.0):
    import torch
    from scann_amd import _native
    xd = torch.from_numpy(x).cuda()
    cd = torch.from_numpy(c).cuda()
    out = torch.empty(x.shape[0], dtype=torch.int32, device="cuda")
    loss = torch.empty(x.shape[0], dtype=torch.float32, device="cuda")
    pd = None if primary is None else torch.from_numpy(primary.astype(np.int32)).cuda()
    _native.nearest_centers_device(xd.data_ptr(), x.shape[0], x.shape[1], cd.data_ptr(),
                                   c.shape[0], out.data_ptr(),
                                   None if pd is None else pd.data_ptr(), lam, loss.data_ptr())
    torch.cuda.synchronize()
    return out.cpu().numpy(), loss.cpu().numpy()


def _check(got, loss64):
    order = np.argsort(loss64, axis=1, kind="stable")
    best = order[:, 0]
    b0 = loss64[np.arange(len(best)), best]
    b1 = loss64[np.arange(len(best)), order[:, 1]]
    clear = (b1 - b0) > 1e-4 * np.maximum(1.0, np.abs(b0))
    assert clear.mean() > 0.9
    np.testing.assert_array_equal(got[clear], best[clear])


@pytest.mark.parametrize("n,d,k", [(5000, 100, 300), (3001, 96, 1000), (777, 2, 16),
                                   (1000, 128, 70)])
def test_kmeans_assignment(n, d, k):
    rng = np.random.default_rng(n + d + k)
    c = rng.standard_normal((k, d)).astype(np.float32)
    x = (c[rng.integers(0, k, n)] + 0.5 * rng.standard_normal((n, d))).astype(np.float32)
    got, _ = _run(x, c)
    x64, c64 = x.astype(np.float64), c.astype(np.float64)
    loss = ((x64[:, None, :] - c64[None, :, :]) ** 2).sum(-1)
    _check(got, loss)


def test_soar_assignment():
    rng = np.random.default_rng(5)
    n, d, k, lam = 4000, 64, 200, 1.5
    c = rng.standard_normal((k, d)).astype(np.float32)
    x = (c[rng.integers(0, k, n)] + 0.4 * rng.standard_normal((n, d))).astype(np.float32)
    x64, c64 = x.astype(np.float64), c.astype(np.float64)
    primary = ((x64[:, None, :] - c64[None]) ** 2).sum(-1).argmin(1)
    got, _ = _run(x, c, primary, lam)
    assert not np.any(got == primary)
    r = x64 - c64[primary]
    diff = x64[:, None, :] - c64[None]
    loss = (diff ** 2).sum(-1) + lam * (np.einsum("nd,nkd->nk", r, diff) ** 2) / \
        np.maximum((r * r).sum(1), 1e-30)[:, None]
    loss[np.arange(n), primary] = np.inf
    _check(got, loss)


def test_builder_uses_the_kernel(monkeypatch):
    """index_builder's assignments run through smx_nearest_centers on a GPU."""
    from scann_amd import _native, index_builder
    calls = []
    real = _native.nearest_centers_device

    def spy(*a, **kw):
        calls.append(a[4])
        return real(*a, **kw)

    monkeypatch.setattr(_native, "nearest_centers_device", spy)
    rng = np.random.default_rng(1)
    x = rng.standard_normal((2000, 16)).astype(np.float32)
    c = index_builder.kmeans(x, 20, 3, seed=0)
    assert c.shape == (20, 16) and len(calls) >= 3


def test_errors():
    from scann_amd import _native
    with pytest.raises(_native.SmxError, match="k > 0"):
        _native.nearest_centers_device(None, 10, 4, None, 0, None)
