"""Generates tests/golden/builder_configs.json from the REFERENCE builder.

Run in the build container only (the reference is not on the GPU box):
    python3 -B tests/golden/make_builder_configs.py
Imports /root/reference/scann/scann_ops/py/scann_builder.py (pure Python,
read-only; -B / dont_write_bytecode keeps the reference tree untouched) and
records the config text it emits for a grid of builder calls.  The fixture is
data (inputs + outputs); tests/test_builder_config.py checks that
scann_amd.scann_builder emits the same parsed config for the same calls.
"""
import importlib.util
import json
import os
import sys

import numpy as np

sys.dont_write_bytecode = True
REF = "/root/reference/scann/scann_ops/py/scann_builder.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "builder_configs.json")

CASES = [
    # (name, db shape, num_neighbors, distance, calls)
    ("glove_tree_ah", (1000, 100), 10, "dot_product",
     [("tree", dict(num_leaves=1000, num_leaves_to_search=100, training_sample_size=250000)),
      ("score_ah", dict(dimensions_per_block=2, anisotropic_quantization_threshold=0.2)),
      ("reorder", dict(reordering_num_neighbors=100))]),
    ("sift_l2", (1000, 128), 10, "squared_l2",
     [("tree", dict(num_leaves=2000, num_leaves_to_search=100)),
      ("score_ah", dict(dimensions_per_block=2)),
      ("reorder", dict(reordering_num_neighbors=100))]),
    ("dot96_soar", (1000, 96), 10, "dot_product",
     [("tree", dict(num_leaves=10000, num_leaves_to_search=150, soar_lambda=1.5,
                    overretrieve_factor=2.0)),
      ("score_ah", dict(dimensions_per_block=2)),
      ("reorder", dict(reordering_num_neighbors=200))]),
    ("odd_dims_no_reorder", (1000, 33), 5, "dot_product",
     [("tree", dict(num_leaves=50, num_leaves_to_search=7, training_iterations=5)),
      ("score_ah", dict(dimensions_per_block=2, training_iterations=4))]),
    ("lut256_l2", (1000, 64), 10, "squared_l2",
     [("tree", dict(num_leaves=100, num_leaves_to_search=10)),
      ("score_ah", dict(dimensions_per_block=4, hash_type="lut256"))]),
    ("brute_force", (1000, 16), 3, "squared_l2",
     [("score_brute_force", dict())]),
    ("dot_tree_nonresidual", (1000, 20), 10, "dot_product",
     [("tree", dict(num_leaves=20, num_leaves_to_search=4, spherical=True,
                    incremental_threshold=0.5)),
      ("score_ah", dict(dimensions_per_block=2, residual_quantization=False)),
      ("reorder", dict(reordering_num_neighbors=40))]),
]


def main():
    spec = importlib.util.spec_from_file_location("ref_scann_builder", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    out = []
    for name, shape, k, dist, calls in CASES:
        b = mod.ScannBuilder(np.zeros(shape, np.float32), k, dist)
        for meth, kw in calls:
            b = getattr(b, meth)(**kw)
        out.append(dict(name=name, shape=list(shape), num_neighbors=k, distance=dist,
                        calls=[[m, kw] for m, kw in calls], config=b.create_config()))
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {len(out)} configs to {OUT}")


if __name__ == "__main__":
    main()
