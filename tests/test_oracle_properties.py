"""Oracle self-consistency at sizes it finishes in seconds.

* the ideal pipeline against an independent exact-arithmetic restatement;
* the AVX2 port (bench.py's cpu_baseline) equals the emulate mode bit for bit;
* emulate-vs-ideal id mismatch stays below the reference's own tolerance
  between its two search modes (1e-3, scann_ops_pybind_test.py:267-278);
* recall against brute force is high (sanity of the whole restatement).
"""
import numpy as np
import pytest

from scann_amd import synthetic
from tests.conftest import make_index
from tests.exact import bits, fadd, ffma, fmul


def _independent_ideal(ix, q, L, k):
    """Exact-rational restatement of pipeline A's pre-reorder stage."""
    from oracle import binding
    out = []
    for qi in range(q.shape[0]):
        scores = []
        for c in range(ix.num_leaves):
            acc = np.float32(0)
            for d in range(ix.dim):
                acc = ffma(-q[qi, d], ix.centers[c, d], acc)
            scores.append((float(acc), c))
        scores.sort()
        leaves = scores[:L]
        _, u8, m = binding.create_lut(q[qi], ix.codebook, 0)
        inv = np.float32(1.0 / np.float64(np.float32(m)))
        shift = 32 - int(np.ceil(np.log2(ix.num_leaves)))
        cands = []
        for bias, leaf in leaves:
            b, e = int(ix.leaf_offsets[leaf]), int(ix.leaf_offsets[leaf + 1])
            for i in range(b, e):
                s = int(u8[np.arange(ix.num_blocks), ix.member_codes[i]].astype(np.int64).sum()) \
                    - 128 * ix.num_blocks
                dd = fadd(fmul(np.float32(s), inv), np.float32(bias))
                cands.append((float(dd), (leaf << shift) | (i - b), int(ix.leaf_members[i])))
        cands.sort(key=lambda t: (t[0], t[1]))
        out.append(sorted(cands[:k], key=lambda t: (t[0], t[2])))
    return out


def test_ideal_matches_exact_restatement(oracle):
    ix, db, q = make_index(n=700, d=8, leaves=9, seed=21, components=12)
    q = q[:4]
    want = _independent_ideal(ix, q, 3, 15)
    gi, gd, gc = oracle.search_pre_reorder(ix, q, 3, 15)
    for r in range(q.shape[0]):
        assert gi[r, :gc[r]].tolist() == [t[2] for t in want[r]]
        assert [bits(x) for x in gd[r, :gc[r]]] == [bits(t[0]) for t in want[r]]


@pytest.mark.parametrize("shared", [True, False])
@pytest.mark.parametrize("reorder", [True, False])
def test_avx2_port_equals_emulate(oracle, small_dot, reorder, shared):
    """Both loop forms of the port (the reference's bottom loop with the
    codes shared by a batch's <= 3 queries, and one pass per query) replay
    the emulate semantics bit for bit."""
    ix, db, q = small_dot
    port = oracle.Avx2Port(ix)
    pi, pd, pc = port.search(q, 12, 100, 10, reorder, 4, batch_shared=shared)
    ei, ed, ec = oracle.search(ix, q, 12, 100, 10, reorder, oracle.MODE_EMULATE)
    np.testing.assert_array_equal(pi, ei)
    np.testing.assert_array_equal(pd.view(np.uint32), ed.view(np.uint32))
    np.testing.assert_array_equal(pc, ec)
    assert set(port.last_phase_s) == {"front", "scan", "tail"}
    assert all(v >= 0.0 for v in port.last_phase_s.values())


def test_emulate_vs_ideal_mismatch_small(oracle):
    ix, db, q = make_index(n=20000, d=32, leaves=64, seed=8, components=100)
    ii, _, _ = oracle.search_pre_reorder(ix, q, 16, 100, oracle.MODE_IDEAL)
    ei, _, _ = oracle.search_pre_reorder(ix, q, 16, 100, oracle.MODE_EMULATE)
    mism = float(np.mean([len(set(a) ^ set(b)) / (2 * len(a)) for a, b in zip(ii, ei)]))
    assert mism < 1e-3


def test_recall_sanity(oracle, small_dot, small_l2):
    for ix, db, q in (small_dot, small_l2):
        gi, _, _ = oracle.search(ix, q, 24, 100, 10, True)
        truth = synthetic.brute_force_topk(db, q, 10, ix.metric)
        assert synthetic.recall_at_k(gi.astype(np.int64), truth, 10) > 0.9


def test_soar_dedupe_and_spilled_members(oracle):
    from scann_amd import index_builder
    db = synthetic.mixture(3000, 16, 32, 0.9, 31)
    q = synthetic.mixture(32, 16, 32, 0.9, 131, means_seed=31)
    ix = index_builder.build_tree_ah(db, 0, 24, 2, training_iterations=4,
                                     ah_training_iterations=4, soar_lambda=1.5)
    assert not ix.disjoint and ix.num_members == 2 * ix.num_datapoints
    gi, gd, gc = oracle.search_pre_reorder(ix, q, 6, 20)
    for r in range(q.shape[0]):
        row = gi[r, :gc[r]].tolist()
        assert len(row) == len(set(row))          # no duplicate ids after dedupe
        assert list(gd[r, :gc[r]]) == sorted(gd[r, :gc[r]])


def _pipeline_b(n=20000, leaves=64, seed=9):
    ix, db, q = make_index(n=n, d=32, leaves=leaves, metric=1, seed=seed, components=100)
    assert not ix.residual
    return ix, db, q


@pytest.mark.parametrize("shared", [True, False])
@pytest.mark.parametrize("reorder", [True, False])
def test_avx2_port_equals_emulate_pipeline_b(oracle, reorder, shared):
    """The port's leaf-major pipeline-B loop (per-leaf int16 top-N merged at
    visit time, tree_x_hybrid_smmd.cc:718-790) equals the oracle's per-query
    replay bit for bit (64 queries x 12 leaves >= 64 leaves: the reference's
    optimized batched path)."""
    ix, db, q = _pipeline_b()
    port = oracle.Avx2Port(ix)
    for nthreads in (1, 4):
        pi, pd, pc = port.search(q, 12, 100, 10, reorder, nthreads, batch_shared=shared)
        ei, ed, ec = oracle.search(ix, q, 12, 100, 10, reorder, oracle.MODE_EMULATE)
        np.testing.assert_array_equal(pi, ei)
        np.testing.assert_array_equal(pd.view(np.uint32), ed.view(np.uint32))
        np.testing.assert_array_equal(pc, ec)


def test_emulate_vs_ideal_pipeline_b(oracle):
    """A.9: pipeline B's emulate result (int16 per-leaf epsilon from the
    global top-k at visit time) against the ideal exact top-k'.  Every
    emulate distance is a genuine candidate distance; the id mismatch stays
    below the reference's tolerance between its search modes (1e-3)."""
    ix, db, q = _pipeline_b()
    ii, idist, ic = oracle.search_pre_reorder(ix, q, 16, 100, oracle.MODE_IDEAL)
    ei, edist, ec = oracle.search_pre_reorder(ix, q, 16, 100, oracle.MODE_EMULATE)
    np.testing.assert_array_equal(ic, ec)
    mism = float(np.mean([len(set(a) ^ set(b)) / (2 * len(a)) for a, b in zip(ii, ei)]))
    assert mism < 1e-3
    # the k'-th distance can only be >= the ideal one
    assert np.all(edist[:, -1] >= idist[:, -1])


def test_emulate_pipeline_b_tight_epsilon(oracle):
    """Many leaves per query and a small k' (frequent GCs and tight int16
    epsilons): emulate still returns k' distinct ids whose distances are the
    LUT16 distances of those ids (checked against the ideal candidate set of
    a wide search)."""
    ix, db, q = _pipeline_b(n=12000, leaves=32, seed=4)
    ei, ed, ec = oracle.search_pre_reorder(ix, q, 32, 5, oracle.MODE_EMULATE)
    wi, wd, wc = oracle.search_pre_reorder(ix, q, 32, 12000, oracle.MODE_IDEAL)
    for r in range(q.shape[0]):
        assert ec[r] == 5 and len(set(ei[r].tolist())) == 5
        lut = dict(zip(wi[r, :wc[r]].tolist(), wd[r, :wc[r]].view(np.uint32).tolist()))
        for i, d in zip(ei[r].tolist(), ed[r].view(np.uint32).tolist()):
            assert lut[i] == d


def test_emulate_pipeline_b_generic_path(oracle):
    """The reference's per-query path for small batches (nq * L < num_leaves,
    tree_x_hybrid_smmd.cc:660-667, 669-691, 875-1028): leaves in top-L
    order, per-leaf int16 FastTopNeighbors, one TopNeighbors<float> per
    query forwarding its approx_bottom.  Against the ideal exact top-k':
    same counts, every emulate distance a genuine LUT16 distance of its id,
    the k'-th never smaller, and the id mismatch below the reference's 1e-3
    tolerance between its search modes."""
    ix, db, q = _pipeline_b()
    for nq, L, k in ((3, 8, 100), (7, 8, 10), (1, 40, 5)):
        assert nq * L < ix.num_leaves          # the generic branch
        qq = q[:nq]
        ii, idist, ic = oracle.search_pre_reorder(ix, qq, L, k, oracle.MODE_IDEAL)
        ei, ed, ec = oracle.search_pre_reorder(ix, qq, L, k, oracle.MODE_EMULATE)
        np.testing.assert_array_equal(ic, ec)
        assert np.all(ed[:, -1] >= idist[:, -1])
        mism = float(np.mean([len(set(a) ^ set(b)) / (2 * len(a)) for a, b in zip(ii, ei)]))
        assert mism < 1e-3
        wi, wd, wc = oracle.search_pre_reorder(ix, qq, L, 20000, oracle.MODE_IDEAL)
        for r in range(nq):
            assert len(set(ei[r].tolist())) == ec[r]
            lut = dict(zip(wi[r, :wc[r]].tolist(), wd[r, :wc[r]].view(np.uint32).tolist()))
            for i, d in zip(ei[r, :ec[r]].tolist(), ed[r, :ec[r]].view(np.uint32).tolist()):
                assert lut[i] == d


def test_emulate_pipeline_b_generic_tight_epsilon(oracle):
    """Generic path with k' = 5 over 32 leaves of one query: the forwarded
    epsilon is the TopNeighbors approx_bottom (not FastTopNeighbors'), so
    later leaves see tight int16 epsilons; results stay k' distinct genuine
    candidates and agree with the ideal top-k' here."""
    ix, db, q = _pipeline_b(n=12000, leaves=64, seed=4)
    qq = q[:1]
    ei, ed, ec = oracle.search_pre_reorder(ix, qq, 32, 5, oracle.MODE_EMULATE)
    ii, idist, ic = oracle.search_pre_reorder(ix, qq, 32, 5, oracle.MODE_IDEAL)
    assert ec[0] == 5 and len(set(ei[0].tolist())) == 5
    assert set(ei[0].tolist()) == set(ii[0].tolist())


def test_emulate_pipeline_b_single_token(oracle):
    """One token on the generic path (L = 1, tree_x_hybrid_smmd.cc:926-949):
    the leaf searcher's own search with pre_reordering_num_neighbors, no
    spilling multiplier and no dedupe; on a SOAR index this is the leaf's
    exact top pre_nn by (int16 distance, id) = the ideal top pre_nn, ids of
    one leaf only."""
    from scann_amd import index_builder, synthetic
    db = synthetic.mixture(5000, 32, 40, 0.6, 9, normalize=False)
    q = synthetic.mixture(4, 32, 40, 0.6, 109, normalize=False, means_seed=9)
    ix = index_builder.build_tree_ah(db, 1, 64, 2, training_iterations=4,
                                     ah_training_iterations=4, soar_lambda=1.5, seed=9)
    assert not ix.residual and not ix.disjoint
    for k in (5, 40):
        ii, idist, ic = oracle.search_pre_reorder(ix, q, 1, k, oracle.MODE_IDEAL)
        ei, ed, ec = oracle.search_pre_reorder(ix, q, 1, k, oracle.MODE_EMULATE)
        np.testing.assert_array_equal(ec, ic)
        assert (ec <= k).all()
        for r in range(q.shape[0]):
            np.testing.assert_array_equal(np.sort(ei[r, :ec[r]]), np.sort(ii[r, :ic[r]]))
