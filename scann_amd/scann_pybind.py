"""``ScannNumpy`` over the MI355X C ABI.

Mirrors the reference's pybind class (scann/scann_ops/cc/scann_npy.{h,cc},
exposed as ``scann_pybind.ScannNumpy`` by scann_pybind.cc:24-54) for the
tree-AH LUT16 path:

* ``ScannNumpy(db, config, training_threads)`` trains an index with
  scann_amd.index_builder and uploads it (scann_npy.cc:67-77);
* ``ScannNumpy(artifacts_dir, assets_pbtxt)`` reloads a serialized searcher
  (scann_npy.cc:57-65) from the reference's artifacts layout
  (scann_amd.assets; an empty ``assets_pbtxt`` reads the directory's
  scann_assets.pbtxt, scann.cc:246-264);
* ``serialize`` writes the reference's layout (scann.cc:504-601,
  scann_npy.cc:272-282);
* ``search`` / ``search_batched`` keep the argument order, the -1 = "config
  default" convention (scann.cc:384-430), the float32 C-order cast, the
  2-D check, the (0, NaN) padding and the x(-1) of dot-product distances
  (scann.h:162-180, scann.cc:364-369).  Errors surface as RuntimeError with
  the reference's "Error during search: " prefix (scann_npy.cc:41-55).
  The search calls run in C++ (``ScannNumpyCore``, scann_amd/csrc/
  smx_pybind.cc, a pybind11 module over the C ABI).
"""
from __future__ import annotations

import ctypes

import os

import numpy as np

from . import _native, assets
from .config import SearchConfig, search_config_from_text
from .index import METRIC_NAMES, TreeAHIndex


def _arg(v) -> int:
    """None means "config default", as -1 does (scann.cc:384-430)."""
    return -1 if v is None else int(v)


def _own_format(directory: str) -> bool:
    """TreeAHIndex.save's layout (smx_index.json + .npy arrays) and no
    reference asset list."""
    return (os.path.isfile(os.path.join(directory, "smx_index.json")) and
            not os.path.isfile(os.path.join(directory, "scann_assets.pbtxt")))


class ScannNumpy:
    def __init__(self, db_or_dir, config: str, training_threads: int = 0, device: int = 0,
                 seed: int = 0):
        if isinstance(db_or_dir, str) and _own_format(db_or_dir):
            # a directory saved by TreeAHIndex.save (this package's own
            # format) with the config text beside it in scann_config.pbtxt
            index = TreeAHIndex.load(db_or_dir)
            if not config:
                with open(os.path.join(db_or_dir, "scann_config.pbtxt")) as f:
                    config = f.read()
            self._cfg = search_config_from_text(config)
        elif isinstance(db_or_dir, str):
            index, tree, self._cfg = assets.load_artifacts(db_or_dir, config or None)
            config = assets.config_text(tree)
        else:
            self._cfg = search_config_from_text(config)
            db = np.ascontiguousarray(db_or_dir, dtype=np.float32)
            if db.ndim != 2:
                raise ValueError("dataset must be two-dimensional")
            from .index_builder import build_tree_ah
            cfg = self._cfg
            index = build_tree_ah(
                db, METRIC_NAMES[cfg.metric], cfg.num_leaves, cfg.dims_per_block,
                training_sample_size=cfg.training_sample_size,
                training_iterations=cfg.training_iterations,
                ah_training_iterations=cfg.ah_training_iterations,
                ah_training_sample_size=cfg.ah_training_sample_size,
                residual=cfg.residual, keep_dataset=cfg.has_reordering,
                soar_lambda=cfg.soar_lambda, overretrieve_factor=cfg.overretrieve_factor,
                seed=seed, noise_shaping_threshold=cfg.noise_shaping_threshold)
        self._config_text = config
        self._index = index
        self._device = device
        self._native = None
        # the search surface in C++ (scann_amd/csrc/smx_pybind.cc): parameter
        # resolution, GIL release, result arrays, x(-1) of dot-product
        # distances (ScannInterface::Initialize) and the error mapping
        cfg = self._cfg
        desc = index.desc()
        self._core = _native.load_pybind().ScannNumpyCore(
            ctypes.addressof(desc), device, cfg.num_neighbors,
            cfg.reorder_num_neighbors if cfg.has_reordering else cfg.num_neighbors,
            cfg.leaves_to_search, cfg.has_reordering, cfg.metric == "dot_product")

    # -- parameter resolution (ScannInterface::GetSearchParameters[Batched]) --
    def _resolve(self, final_nn: int, pre_reorder_nn: int, leaves: int):
        cfg = self._cfg
        final_nn = cfg.num_neighbors if final_nn is None or final_nn <= 0 else int(final_nn)
        if cfg.has_reordering:
            pre = cfg.reorder_num_neighbors if pre_reorder_nn is None or pre_reorder_nn <= 0 \
                else int(pre_reorder_nn)
        else:
            pre = final_nn
        leaves = cfg.leaves_to_search if leaves is None or leaves <= 0 else int(leaves)
        return final_nn, pre, leaves

    def search(self, query, final_nn=-1, pre_reorder_nn=-1, leaves=-1):
        """ScannNumpy::Search: one query through the single-query path's
        numerics (one-to-many partition scores, smx_search)."""
        return self._core.search(query, _arg(final_nn), _arg(pre_reorder_nn), _arg(leaves))

    def search_batched(self, queries, final_nn=-1, pre_reorder_nn=-1, leaves=-1,
                       parallel=False, batch_size=256):
        # parallel mode (SearchBatchedParallel) exists to spread a batch over
        # CPU threads; the GPU batch is already parallel, so both modes run
        # the same device pipeline (results identical by construction).
        return self._core.search_batched(queries, _arg(final_nn), _arg(pre_reorder_nn),
                                         _arg(leaves), bool(parallel), int(batch_size or 0))

    def serialize(self, path: str, relative_path: bool = False) -> None:
        try:
            assets.save_artifacts(self._index, self._config_text, path, relative_path)
        except (OSError, ValueError) as e:
            raise RuntimeError(f"Failed to extract SingleMachineFactoryOptions: {e}") from None

    def config(self) -> str:
        return self._config_text

    def size(self) -> int:
        return self._index.num_datapoints

    def set_num_threads(self, num_threads: int) -> None:
        del num_threads  # host threads do not drive the GPU pipeline

    def native(self) -> _native.NativeIndex:
        """A ctypes handle on its own device copy of the index (stage entry
        points, tuning); created on first use."""
        if self._native is None:
            self._native = _native.NativeIndex(self._index, device=self._device)
        return self._native

    @property
    def index(self) -> TreeAHIndex:
        return self._index
