"""The seed threshold select (smx_kth_threshold_keys) against numpy.

A query's scan prunes with the kk-th smallest of its seed distances (the
first leaves' order-preserving distance bits), the bound the reference's
TopNeighbors keeps while it scans (scann/utils/fast_top_neighbors.h).  The
device select (ThresholdOfVals: a block rank of the 256 per-thread minima,
then an exact rank of the values under that bound, or histogram rounds) must
return exactly (v << 32) | 0xFFFFFFFF for v the kk-th smallest value, and ~0
when a set holds fewer than kk values.  Bit-exact: integer work.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

KEYS = 4096
NONE = 0xFFFFFFFF


def _expected(sets, kk):
    out = np.empty(sets.shape[0], dtype=np.uint64)
    for i, s in enumerate(sets):
        v = np.sort(s[s != NONE])
        out[i] = (np.uint64(v[kk - 1]) << np.uint64(32)) | np.uint64(NONE) \
            if kk > 0 and v.size >= kk else np.uint64(~np.uint64(0))
    return out


def _device(sets, kk):
    from scann_amd import _native
    d = torch.from_numpy(sets.view(np.int32).copy()).cuda()
    o = torch.empty(sets.shape[0], dtype=torch.int64, device="cuda")
    _native.kth_threshold_keys_device(d.data_ptr(), sets.shape[0], kk, o.data_ptr())
    torch.cuda.synchronize()
    return o.cpu().numpy().view(np.uint64)


def _sets(rng, kind, n):
    s = np.full((n, KEYS), NONE, dtype=np.uint32)
    for i in range(n):
        if kind == "uniform":
            s[i] = rng.integers(0, NONE, KEYS, dtype=np.uint32)
        elif kind == "clustered":        # a narrow band: ties in the top bits
            s[i] = 0x9F000000 + rng.integers(0, 5000, KEYS, dtype=np.uint32)
        elif kind == "ties":              # few distinct values
            s[i] = rng.choice(np.array([7, 9, 9, 12, 0xFFFFFFFE], np.uint32), KEYS)
        elif kind == "equal":
            s[i] = 0x80001234
        elif kind == "ragged":            # a prefix of real values, the rest none
            m = int(rng.integers(0, KEYS + 1))
            s[i, :m] = rng.integers(0x80000000, 0x80100000, m, dtype=np.uint32)
        elif kind == "one_thread":        # values in one thread's 16 slots only
            s[i, 5::256] = rng.integers(100, 200, 16, dtype=np.uint32)
        elif kind == "sorted_desc":
            s[i] = np.sort(rng.integers(0, 1 << 31, KEYS, dtype=np.uint32))[::-1]
    return s


@pytest.mark.parametrize("kind", ["uniform", "clustered", "ties", "equal", "ragged",
                                  "one_thread", "sorted_desc"])
@pytest.mark.parametrize("kk", [1, 10, 100, 200, 256, 257, 512, 1000, 4096])
def test_kth_threshold_keys(kind, kk):
    rng = np.random.default_rng(kk * 31 + len(kind))
    sets = _sets(rng, kind, 48)
    np.testing.assert_array_equal(_device(sets, kk), _expected(sets, kk),
                                  err_msg=f"{kind} kk={kk}")


def test_kth_threshold_keys_fewer_values_than_kk():
    s = np.full((3, KEYS), NONE, dtype=np.uint32)
    s[0, :99] = 5
    s[1, :100] = np.arange(100, dtype=np.uint32)
    got = _device(s, 100)
    assert got[0] == np.uint64(~np.uint64(0)) and got[2] == np.uint64(~np.uint64(0))
    assert got[1] == (np.uint64(99) << np.uint64(32)) | np.uint64(NONE)
    assert (_device(s, 0) == np.uint64(~np.uint64(0))).all()
