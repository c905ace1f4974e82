"""The on-device generator of BASELINE configs 4/5 (scann_amd/generate.py):
chunks regenerate bit for bit (CPU), and -- on the GPU, where the build's HIP
kernels run -- the W shards a rank-by-rank build produces are exactly the
range split of the whole index (members of every leaf contiguous from
leaf_row_base, identical codes, whole-index shift)."""
import numpy as np
import pytest
import torch

from scann_amd import generate


def _ds(n=150_000, dim=24, seed=4, device="cpu"):
    return generate.GeneratedDataset(n, dim, seed, components=64, device=torch.device(device))


def test_chunks_regenerate_and_rows_are_unit():
    ds = _ds()
    a = ds.rows(70_000, 5000)
    b = _ds().rows(65_536, 10_000)[70_000 - 65_536:70_000 - 65_536 + 5000]
    assert torch.equal(a, b)
    assert torch.allclose(a.norm(dim=1), torch.ones(5000), atol=1e-5)
    assert ds.num_chunks == 3


@pytest.mark.gpu
@pytest.mark.parametrize("soar", [None, 1.5])
def test_rank_shards_are_the_range_split_of_the_whole_index(soar):
    ds = _ds(device="cuda")
    kw = dict(soar_lambda=soar, training_sample_size=20_000, training_iterations=3,
              ah_training_sample_size=10_000, ah_training_iterations=3, seed=1)
    whole = generate.build_generated_shard(ds, 40, 0, 1, **kw)
    assert whole.num_members == (2 if soar else 1) * ds.n
    shards = [generate.build_generated_shard(ds, 40, r, 3, **kw) for r in range(3)]
    wo = whole.leaf_offsets.astype(np.int64)
    for sh in shards:
        assert sh.is_shard and sh.global_topn_shift == whole.global_topn_shift_value()
        assert sh.disjoint == whole.disjoint
    for leaf in range(whole.num_leaves):
        got_m, got_c = [], []
        for sh in shards:
            so = sh.leaf_offsets.astype(np.int64)
            assert int(sh.leaf_row_base[leaf]) == len(got_m)
            got_m += sh.leaf_members[so[leaf]:so[leaf + 1]].tolist()
            got_c.append(sh.member_codes[so[leaf]:so[leaf + 1]])
        assert got_m == whole.leaf_members[wo[leaf]:wo[leaf + 1]].tolist()
        np.testing.assert_array_equal(np.concatenate(got_c),
                                      whole.member_codes[wo[leaf]:wo[leaf + 1]])
    # the shard carries its members' float rows for the reorder
    sh = shards[1]
    np.testing.assert_array_equal(sh.member_rows, whole.dataset[sh.leaf_members])


@pytest.mark.gpu
def test_rank_without_chunks_is_an_empty_shard():
    ds = _ds(n=100_000, device="cuda")   # 2 chunks, 3 ranks
    sh = generate.build_generated_shard(ds, 8, 0, 3, training_sample_size=5000,
                                        training_iterations=2, ah_training_sample_size=5000,
                                        ah_training_iterations=2)
    assert sh.num_members == 0 and sh.is_shard
