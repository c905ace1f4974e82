"""Hand-derived known-answer tests pinning the CPU oracle to the reference's
semantics.  The reference ships no golden vectors for
this path and cannot be built here, so these KATs -- values
derived by hand or by exact rational arithmetic from the cited formulas --
are the oracle's pins.
"""
import numpy as np
import pytest

from scann_amd.index import TreeAHIndex
from tests.exact import bits, fadd, ffma, fmul, fsub


def test_partition_dot_is_fma_chain(oracle):
    """many_to_many_impl.inc:544-556: acc <- fma(-q_d, c_d, acc) from 0."""
    rng = np.random.default_rng(1)
    q = rng.standard_normal((3, 11)).astype(np.float32)
    c = rng.standard_normal((5, 11)).astype(np.float32)
    got = oracle.partition_scores(q, c, 0)
    for i in range(3):
        for j in range(5):
            acc = np.float32(0)
            for d in range(11):
                acc = ffma(-q[i, d], c[j, d], acc)
            assert bits(got[i, j]) == bits(acc)


def test_partition_topl_ties_by_center_index(oracle):
    """Equal scores keep the lower center index (CompIV, fast_top_neighbors.cc:96-105)."""
    q = np.array([[1.0, 0.0]], np.float32)
    c = np.array([[0.5, 1.0], [0.25, 0.0], [0.5, -1.0], [0.5, 3.0]], np.float32)
    leaf, score = oracle.partition_topl(q, c, 0, 3)
    assert leaf.tolist() == [[0, 2, 3]]
    assert score.tolist() == [[-0.5, -0.5, -0.5]]


def test_raw_lut_two_dim_block_is_unfused(oracle):
    """A.2: LUT[b][c] = -fl(fl(q0*c0) + fl(q1*c1))."""
    rng = np.random.default_rng(2)
    q = rng.standard_normal(6).astype(np.float32)
    cb = rng.standard_normal((3, 16, 2)).astype(np.float32)
    raw, _, _ = oracle.create_lut(q, cb, 0)
    for b in range(3):
        for k in range(16):
            want = -fadd(fmul(q[2 * b], cb[b, k, 0]), fmul(q[2 * b + 1], cb[b, k, 1]))
            assert bits(raw[b, k]) == bits(want)


def test_raw_lut_squared_l2_and_partial_block(oracle):
    """A.9: fl(fl(t0*t0) + fl(t1*t1)), t = fl(q - c); a 1-dim last block."""
    rng = np.random.default_rng(3)
    q = rng.standard_normal(5).astype(np.float32)
    cb = rng.standard_normal((3, 16, 2)).astype(np.float32)
    raw, _, _ = oracle.create_lut(q, cb, 1)
    for b in range(3):
        for k in range(16):
            t0 = fsub(q[2 * b], cb[b, k, 0])
            if b < 2:
                t1 = fsub(q[2 * b + 1], cb[b, k, 1])
                want = fadd(fmul(t0, t0), fmul(t1, t1))
            else:
                want = fmul(t0, t0)
            assert bits(raw[b, k]) == bits(want)


def test_fixed_point_conversion_by_hand(oracle):
    """A.3: m = 127 / max|LUT|; u8 = round_half_away(LUT * m) + 128.

    Query (1, 0) per block makes LUT[b][k] = -c0 exactly.  With max|LUT| = 2:
    m = 63.5; LUT -2 -> -127 -> 1; +1 -> 63.5 -> 64 -> 192 (half away from
    zero); -0.5 -> -31.75 -> -32 -> 96; -0.25 -> -15.875 -> -16 -> 112;
    0 -> 128; +0.0078125 -> 0.49609375 -> 0 -> 128.
    """
    c0 = np.array([2.0, -1.0, 0.5, 0.25, 0.0, -0.0078125] + [0.0] * 10, np.float32)
    cb = np.zeros((1, 16, 2), np.float32)
    cb[0, :, 0] = c0
    cb[0, :, 1] = 7.0  # multiplied by q1 = 0
    raw, u8, m = oracle.create_lut(np.array([1.0, 0.0], np.float32), cb, 0)
    assert m == 63.5
    assert u8[0, :6].tolist() == [1, 192, 96, 112, 128, 128]


def test_fixed_point_floor_for_tiny_tables(oracle):
    """max|LUT| below sqrt(FLT_EPSILON) uses that floor (asymmetric_hashing_impl.cc:575)."""
    cb = np.zeros((1, 16, 2), np.float32)
    _, u8, m = oracle.create_lut(np.array([1.0, 0.0], np.float32), cb, 0)
    assert np.float32(m) == np.float32(127.0) / np.sqrt(np.finfo(np.float32).eps)
    assert (u8 == 128).all()


def _codes33():
    return np.array([[(i * 5 + b * 3) % 16 for b in range(3)] for i in range(33)], np.uint8)


def test_packed_layout_by_hand(oracle):
    """asymmetric_hashing_impl.cc:690-737: byte[g*16B + b*16 + m] =
    code[32g+16+m][b] << 4 | code[32g+m][b]; the tail repeats the last point."""
    p = oracle.pack_codes(_codes33())
    assert p.size == 3 * 64 // 2
    assert p[0] == 0x00 and p[1] == 0x55 and p[2] == 0xAA   # group 0, block 0
    assert p[16] == 0x33                                     # block 1, m = 0
    assert p[48] == 0x00                                     # group 1, block 0, m = 0
    assert p[48 + 32 + 1] == 0x66                            # group 1, block 2, m = 1 (clamped)


def test_lut16_accumulation_by_hand(oracle):
    """A.4: acc = sum_b (u8[b][code] - 128), exact in int."""
    lut = np.array([[128 + (k - 8) * (b + 1) for k in range(16)] for b in range(3)], np.uint8)
    acc = oracle.lut16_accumulate(oracle.pack_codes(_codes33()), 33, 3, lut)
    # dp 0: codes (0, 3, 6) -> -8*1 + -5*2 + -2*3 = -24
    # dp 32: codes (0, 3, 6) as well (32*5 % 16 = 0)
    assert acc[0] == -24 and acc[32] == -24
    # dp 1: codes (5, 8, 11) -> -3*1 + 0*2 + 3*3 = 6
    assert acc[1] == 6
    codes = _codes33().astype(np.int64)
    want = ((codes - 8) * np.array([1, 2, 3])).sum(1)
    np.testing.assert_array_equal(acc, want)


def _toy_index(dataset=True):
    """2 leaves, 3 blocks of 2 dims; hand-chosen codes and centers."""
    cb = np.zeros((3, 16, 2), np.float32)
    for b in range(3):
        for k in range(16):
            cb[b, k] = ((k - 8) * 0.125 * (b + 1), (k % 3) * 0.25)
    codes = _codes33()
    centers = np.array([[0.5, 0, 0, 0, 0, 0], [-0.25, 0.5, 0, 0, 0.125, 0]], np.float32)
    offsets = np.array([0, 20, 33], np.uint64)
    members = np.arange(33, dtype=np.uint32)
    ds = np.random.default_rng(4).standard_normal((33, 6)).astype(np.float32) if dataset else None
    return TreeAHIndex(metric=0, dim=6, num_blocks=3, dims_per_block=2, residual=True,
                       centers=centers, codebook=cb, leaf_offsets=offsets, leaf_members=members,
                       member_codes=codes, num_datapoints=33, dataset=ds)


def test_toy_index_distances_follow_a5(oracle):
    """A.5: d = fl(fl(float(acc) * inv) + bias), inv = float(1.0 / double(m)),
    bias = the dot FMA chain; ideal top-k by (d, packed id); output sorted by
    (d, global id)."""
    ix = _toy_index()
    q = np.array([0.75, -0.5, 0.25, 1.0, -0.125, 0.5], np.float32)
    assert oracle.global_topn_shift(ix) == 31
    _, u8, m = oracle.create_lut(q, ix.codebook, 0)
    inv = np.float32(1.0 / np.float64(np.float32(m)))
    biases = []
    for leaf in range(2):
        acc = np.float32(0)
        for d in range(6):
            acc = ffma(-q[d], ix.centers[leaf, d], acc)
        biases.append(acc)
    cands = []
    for leaf in range(2):
        b, e = int(ix.leaf_offsets[leaf]), int(ix.leaf_offsets[leaf + 1])
        for i in range(b, e):
            s = sum(int(u8[blk, ix.member_codes[i, blk]]) - 128 for blk in range(3))
            d = fadd(fmul(np.float32(s), inv), biases[leaf])
            cands.append((float(d), (leaf << 31) | (i - b), i))
    cands.sort(key=lambda t: (t[0], t[1]))
    top = sorted(cands[:7], key=lambda t: (t[0], t[2]))
    gi, gd, gc = oracle.search_pre_reorder(ix, q[None, :], 2, 7)
    assert gc[0] == 7
    assert gi[0].tolist() == [t[2] for t in top]
    assert [bits(x) for x in gd[0]] == [bits(t[0]) for t in top]


def test_exact_reorder_distance_a8(oracle):
    """A.8 for D = 13: 8 fused lanes, fold (l, l+4), 4-wide step, tail."""
    rng = np.random.default_rng(5)
    q = rng.standard_normal(13).astype(np.float32)
    x = rng.standard_normal(13).astype(np.float32)
    a = [ffma(-q[l], x[l], np.float32(0)) for l in range(8)]
    s = [fadd(a[l + 4], a[l]) for l in range(4)]
    s = [ffma(-q[8 + l], x[8 + l], s[l]) for l in range(4)]
    r = fadd(fadd(s[0], s[2]), fadd(s[1], s[3]))
    r = ffma(-q[12], x[12], r)
    assert bits(oracle.exact_distance(q, x, 0)) == bits(r)
    # squared L2 with the 2-wide (lanes 2, 3) step: D = 10
    q2, x2 = q[:10], x[:10]
    t = [fsub(q2[l], x2[l]) for l in range(10)]
    a = [ffma(t[l], t[l], np.float32(0)) for l in range(8)]
    s = [fadd(a[l + 4], a[l]) for l in range(4)]
    s[2] = ffma(t[8], t[8], s[2])
    s[3] = ffma(t[9], t[9], s[3])
    r = fadd(fadd(s[0], s[2]), fadd(s[1], s[3]))
    assert bits(oracle.exact_distance(q2, x2, 1)) == bits(r)


def test_fast_topn_replay_exact_after_gc(oracle):
    """A.6: buffered top-N with approximate GC ends with the exact top-k by (d, id)."""
    rng = np.random.default_rng(6)
    ids = np.arange(200, dtype=np.uint32)
    d = rng.standard_normal(200).astype(np.float32)
    oi, od, ngc = oracle.fast_topn_replay(ids, d, 20)
    order = np.lexsort((ids, d))[:20]
    assert oi.tolist() == ids[order].tolist()
    assert ngc >= 1


@pytest.mark.parametrize("k,n,span,eps", [(20, 600, 12, 32767), (100, 3000, 40, 32767),
                                          (7, 500, 5, 3), (150, 2000, 400, 300)])
def test_fast_topn_int16_replay_exact_set(oracle, k, n, span, eps):
    """Pipeline B's per-leaf FastTopNeighbors<int16_t> (querying.h:403-462):
    ids pushed in ascending order (local datapoint order), heavy ties; the
    finished set is the exact top-k by (value, id) of the values < eps, the
    GC (with the two-stream DoublePorted compaction) having run."""
    rng = np.random.default_rng(k + n)
    ids = np.arange(n, dtype=np.uint32)
    d = rng.integers(0, span, n).astype(np.int16)
    oi, od, ngc = oracle.fast_topn_replay_i16(ids, d, k, eps)
    keep = d < eps
    order = np.lexsort((ids[keep], d[keep]))[:k]
    assert sorted(zip(od.tolist(), oi.tolist())) == \
        sorted(zip(d[keep][order].tolist(), ids[keep][order].tolist()))
    if keep.sum() >= 2 * k:
        assert ngc >= 1
