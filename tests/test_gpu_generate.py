"""configs[3]/[4] as bench.py builds them: shards generated rank by rank on
the GPU (scann_amd/generate.py), searched and merged == the whole generated
index searched on the GPU == the ideal oracle."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("soar,leaves,world", [(1.5, 600, 4), (None, 2000, 8)])
def test_generated_shards_merge_to_the_whole_index(oracle, soar, leaves, world):
    from scann_amd import _native, generate
    from scann_amd.distributed import NativeShardEngine
    ds = generate.GeneratedDataset(500_000, 96, 4, device=torch.device("cuda"))
    kw = dict(soar_lambda=soar, training_sample_size=60_000, training_iterations=4,
              ah_training_sample_size=40_000, ah_training_iterations=4, seed=4)
    whole = generate.build_generated_shard(ds, leaves, 0, 1, **kw)
    q = ds.queries(256, 99)
    nat = _native.NativeIndex(whole)
    wi, wd, wc = nat.search_batched(q, 40, 100, 10, True)
    oi, od, oc = oracle.search(whole, q[:64], 40, 100, 10, True, oracle.MODE_IDEAL, 16)
    np.testing.assert_array_equal(wi[:64], oi)
    np.testing.assert_array_equal(wd[:64].view(np.uint32), od.view(np.uint32))
    nat.close()
    engines = [NativeShardEngine(generate.build_generated_shard(ds, leaves, r, world, **kw))
               for r in range(world)]
    qd = torch.from_numpy(q).cuda()
    k = engines[0].shard_width(40, 100, 10, True)
    ent = torch.empty((world, q.shape[0], k, 2), dtype=torch.int64, device="cuda")
    for r, e in enumerate(engines):
        e.search_shard(qd, 40, 100, 10, True, ent[r])
    si, sd, sc = engines[0].merge(world, ent, q.shape[0], 40, 100, 10, True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(si.cpu().numpy().astype(np.uint32), wi)
    np.testing.assert_array_equal(sd.cpu().numpy().view(np.uint32), wd.view(np.uint32))
    np.testing.assert_array_equal(sc.cpu().numpy(), wc)
    for e in engines:
        e.nat.close()
