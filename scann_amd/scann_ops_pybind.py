"""Python surface of the reference's scann_ops_pybind module
(scann/scann_ops/py/scann_ops_pybind.py:38-273), backed by the MI355X path.

    searcher = scann_ops_pybind.builder(db, 10, "dot_product").tree(
        num_leaves=1000, num_leaves_to_search=100).score_ah(2).reorder(100).build()
    neighbors, distances = searcher.search_batched(queries)

Out of scope for this tier: online mutation (upsert,
delete, rebalance, reserve), health stats and autopilot; they raise
NotImplementedError rather than silently doing nothing.
"""
from __future__ import annotations

import json
import os

import numpy as np

from . import scann_builder
from .scann_pybind import ScannNumpy


class ScannSearcher:
    """Wrapper class around ScannNumpy that provides a cleaner interface."""

    def __init__(self, searcher, docids=None):
        self.searcher = searcher
        self.docids = docids
        if docids is not None:
            self.docid_to_id = {docid: i for i, docid in enumerate(docids)}
            if len(docids) != len(self.docid_to_id):
                raise ValueError("Duplicates found in docids.")

    def search(self, q, final_num_neighbors=-1, pre_reorder_num_neighbors=-1,
               leaves_to_search=-1):
        """Single-query search; -1 for a param uses the searcher's default value."""
        idx, dist = self.searcher.search(q, final_num_neighbors, pre_reorder_num_neighbors,
                                         leaves_to_search)
        idx = idx if self.docids is None else [self.docids[j] for j in idx]
        return idx, dist

    def search_batched(self, queries, final_num_neighbors=None, pre_reorder_num_neighbors=None,
                       leaves_to_search=None):
        """Search method for multiple queries."""
        final_nn = -1 if final_num_neighbors is None else final_num_neighbors
        pre_nn = -1 if pre_reorder_num_neighbors is None else pre_reorder_num_neighbors
        leaves = -1 if leaves_to_search is None else leaves_to_search
        idx, dist = self.searcher.search_batched(queries, final_nn, pre_nn, leaves, False, 0)
        if self.docids is not None:
            idx = [[self.docids[j] for j in row] for row in idx]
        return idx, dist

    def search_batched_parallel(self, queries, final_num_neighbors=None,
                                pre_reorder_num_neighbors=None, leaves_to_search=None,
                                batch_size=256):
        """Search method for multiple queries with multiple threads."""
        final_nn = -1 if final_num_neighbors is None else final_num_neighbors
        pre_nn = -1 if pre_reorder_num_neighbors is None else pre_reorder_num_neighbors
        leaves = -1 if leaves_to_search is None else leaves_to_search
        idx, dist = self.searcher.search_batched(queries, final_nn, pre_nn, leaves, True,
                                                 batch_size)
        if self.docids is not None:
            idx = [[self.docids[j] for j in row] for row in idx]
        return idx, dist

    def serialize(self, artifacts_dir, relative_path=False):
        self.searcher.serialize(artifacts_dir, relative_path)
        if self.docids is not None:
            # JSON, not pickle: loading must not execute anything from the file.
            with open(os.path.join(artifacts_dir, "scann_docids.json"), "w") as f:
                json.dump(list(self.docids), f)

    def size(self):
        return self.searcher.size()

    def set_num_threads(self, num_threads):
        self.searcher.set_num_threads(num_threads)

    def config(self):
        return self.searcher.config()

    def _unsupported(self, *args, **kwargs):
        raise NotImplementedError(
            "online mutation / health stats are outside the MI355X tree-AH query path")

    upsert = delete = rebalance = reserve = _unsupported
    get_health_stats = initialize_health_stats = _unsupported


def builder(db, num_neighbors, distance_measure):
    """pybind analogue of builder() in scann_ops.py."""

    class ScannBuilder(scann_builder.ScannBuilder):
        def create_config(self):
            if self.params.get("autopilot") is not None:
                raise NotImplementedError("autopilot is outside the MI355X tree-AH query path")
            return super().create_config()

    def builder_lambda(db, config, training_threads, **kwargs):
        return create_searcher(db, config, training_threads, **kwargs)

    return ScannBuilder(db, num_neighbors, distance_measure).set_builder_lambda(builder_lambda)


def create_searcher(db, scann_config, training_threads=0, docids=None, **kwargs):
    """Creates a searcher object wrapping a ScannNumpy object."""
    if docids is not None and len(docids) != db.shape[0]:
        raise ValueError(f"docid and database size mismatch: {len(docids)} != {db.shape[0]}.")
    if isinstance(db, np.ndarray) and db.shape[0] == 0:
        raise ValueError("an empty database cannot be partitioned (dynamic config is out of scope)")
    device = kwargs.pop("device", 0)
    seed = kwargs.pop("seed", 0)
    return ScannSearcher(ScannNumpy(db, scann_config, training_threads, device=device, seed=seed),
                         docids=docids)


def load_searcher(artifacts_dir, assets_backcompat_shim=True, device=0):
    """Loads searcher assets from artifacts_dir and returns a ScaNN searcher
    (scann_ops_pybind.py:250-270 of the reference).  Without a
    scann_assets.pbtxt the backcompat shim lists the asset files present
    (scann_ops_pybind_backcompat.py:30-70) and writes that list."""
    if not os.path.isdir(artifacts_dir):
        raise ValueError(f"{artifacts_dir} is not a directory.")
    own = os.path.join(artifacts_dir, "smx_index.json")
    assets_pbtxt = os.path.join(artifacts_dir, "scann_assets.pbtxt")
    if os.path.isfile(own) and not os.path.isfile(assets_pbtxt):
        # this package's own format (TreeAHIndex.save) + scann_config.pbtxt
        cfg = os.path.join(artifacts_dir, "scann_config.pbtxt")
        if not os.path.isfile(cfg):
            raise ValueError(f"{artifacts_dir}: smx_index.json needs scann_config.pbtxt beside it")
        with open(cfg) as f:
            return ScannSearcher(ScannNumpy(artifacts_dir, f.read(), device=device))
    if not os.path.exists(assets_pbtxt):
        if not assets_backcompat_shim:
            raise ValueError("No scann_assets.pbtxt found.")
        _populate_and_save_assets_proto(artifacts_dir)
    docids = None
    p = os.path.join(artifacts_dir, "scann_docids.json")
    if os.path.isfile(p):
        with open(p) as f:
            docids = json.load(f)
    elif os.path.isfile(os.path.join(artifacts_dir, "scann_docids.pkl")):
        # loading a pickle executes code from the file; never done here
        raise ValueError("scann_docids.pkl is a pickle and is not loaded; "
                         "convert the docids to scann_docids.json (a JSON list)")
    with open(assets_pbtxt) as f:
        return ScannSearcher(ScannNumpy(artifacts_dir, f.read(), device=device), docids)


_BACKCOMPAT_ASSETS = (
    ("ah_codebook.pb", "AH_CENTERS"), ("serialized_partitioner.pb", "PARTITIONER"),
    ("datapoint_to_token.npy", "TOKENIZATION_NPY"), ("hashed_dataset.npy", "AH_DATASET_NPY"),
    ("int8_dataset.npy", "INT8_DATASET_NPY"), ("int8_multipliers.npy", "INT8_MULTIPLIERS_NPY"),
    ("dp_norms.npy", "INT8_NORMS_NPY"), ("dataset.npy", "DATASET_NPY"))


def _populate_and_save_assets_proto(artifacts_dir):
    from .assets import format_message
    found = [{"asset_type": [kind], "asset_path": [os.path.join(artifacts_dir, name)]}
             for name, kind in _BACKCOMPAT_ASSETS
             if os.path.exists(os.path.join(artifacts_dir, name))]
    with open(os.path.join(artifacts_dir, "scann_assets.pbtxt"), "w") as f:
        f.write(format_message({"assets": found}, "ScannAssets"))
