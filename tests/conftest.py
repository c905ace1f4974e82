import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libscann_mi355x.so)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import binding
    binding.build()
    return binding


def make_index(n=6000, d=32, leaves=48, dpb=2, metric=0, seed=11, components=64,
               spread=0.9, keep_dataset=True):
    from scann_amd import index_builder, synthetic
    normalize = metric == 0
    db = synthetic.mixture(n, d, components, spread, seed, normalize=normalize)
    q = synthetic.mixture(64, d, components, spread, seed + 100, normalize=normalize,
                          means_seed=seed)
    ix = index_builder.build_tree_ah(db, metric, leaves, dpb, training_iterations=6,
                                     ah_training_iterations=6, keep_dataset=keep_dataset,
                                     seed=seed)
    return ix, db, q


@pytest.fixture(scope="session")
def small_dot():
    return make_index()


@pytest.fixture(scope="session")
def small_l2():
    return make_index(metric=1, seed=5)
