"""Fluent builder with the reference's API (scann/scann_ops/py/scann_builder.py).

Same method names, argument names, defaults and error behaviour as the
reference's ``ScannBuilder``; ``create_config`` emits a ScannConfig text proto
with the same fields (tests/golden/builder_configs.json holds configs the
reference builder produced, and tests/test_builder_config.py compares the
parsed trees).  Which configs the MI355X searcher accepts is decided in
scann_amd.config.search_config_from_text.
"""
from __future__ import annotations

import enum
import functools
import inspect


class ReorderType(enum.Enum):
    FLOAT32 = 1
    INT8 = 2
    BFLOAT16 = 3


class IncrementalMode(enum.Enum):
    NONE = 1
    ONLINE = 2
    ONLINE_INCREMENTAL = 3


def _stanza(key):
    """Records a configuration step; the stanza text is produced at
    create_config time by the wrapped function (scann_builder.py:22-37)."""

    def wrap(fn):
        sig = inspect.signature(fn)

        @functools.wraps(fn)
        def record(self, *args, **kwargs):
            if key in self.params:
                raise Exception(f"{key} has already been configured")
            bound = sig.bind_partial(self, *args, **kwargs)
            params = dict(bound.arguments)
            params.pop("self")
            self.params[key] = params
            return self

        record.proto_maker = fn
        return record

    return wrap


def _b(v) -> str:
    return "True" if v else "False"


def _quant_name(q) -> str:
    if q is True:
        q = ReorderType.INT8
    elif q is False:
        q = ReorderType.FLOAT32
    return {ReorderType.INT8: "FIXED8", ReorderType.BFLOAT16: "BFLOAT16",
            ReorderType.FLOAT32: "FLOAT32"}[q]


def _as_reorder_type(q):
    if q is True:
        return ReorderType.INT8
    if q is False:
        return ReorderType.FLOAT32
    return q


class ScannBuilder:
    """See the reference's ScannBuilder for the meaning of every option."""

    def __init__(self, db, num_neighbors, distance_measure):
        self.params = {}
        self.training_threads = 0
        self.builder_lambda = None
        self.db = db
        self.num_neighbors = num_neighbors
        self.distance_measure = distance_measure

    def set_n_training_threads(self, threads):
        self.training_threads = threads
        return self

    def set_builder_lambda(self, builder_lambda):
        self.builder_lambda = builder_lambda
        return self

    # -- projection stanzas -------------------------------------------------
    @_stanza("pca")
    def pca(self, reduction_dim=None, pca_significance_threshold=0.80,
            pca_truncation_threshold=0.6):
        dim = self.db.shape[1]
        if reduction_dim is not None and pca_significance_threshold is None:
            body = f"num_dims_per_block: {reduction_dim}"
        elif pca_significance_threshold is not None and reduction_dim is None:
            body = (f"pca_significance_threshold: {pca_significance_threshold}\n"
                    f"pca_truncation_threshold: {pca_truncation_threshold}")
        else:
            raise ValueError("pca must be called with either reduction_dim or "
                             "pca_significance_threshold")
        return f"projection: {{\n projection_type: PCA\n input_dim: {dim}\n {body}\n}}"

    @_stanza("truncate")
    def truncate(self, reduction_dim):
        dim = self.db.shape[1]
        if reduction_dim >= dim:
            raise ValueError(f"reduction_dim must be less than {dim}")
        return (f"projection: {{\n projection_type: TRUNCATE\n num_dims_per_block: "
                f"{reduction_dim}\n input_dim: {dim}\n}}")

    # -- partitioning -------------------------------------------------------
    @_stanza("upper_tree")
    def upper_tree(self, num_leaves, num_leaves_to_search, avq=float("nan"), soar_lambda=None,
                   overretrieve_factor=None, scoring_mode=ReorderType.INT8,
                   anisotropic_quantization_threshold=float("nan")):
        return "\n".join([
            "enabled: true",
            f"num_centroids: {num_leaves}",
            f"num_centroids_to_search: {num_leaves_to_search}",
            f"avq: {avq}",
            f"soar: {{ enabled: {soar_lambda is not None} lambda: {soar_lambda or 1.5} "
            f"overretrieve_factor: {overretrieve_factor or 2.0} }}",
            f"quantization: {_quant_name(scoring_mode)}",
            f"noise_shaping_threshold: {anisotropic_quantization_threshold}",
        ])

    @_stanza("tree")
    def tree(self, num_leaves, num_leaves_to_search, training_sample_size=100000,
             min_partition_size=50, training_iterations=12, spherical=False,
             quantize_centroids=False, random_init=True, incremental_threshold=None, avq=None,
             soar_lambda=None, overretrieve_factor=None, distance_measure=None,
             projection=None, upper_tree=None):
        lines = [
            f"num_children: {num_leaves}",
            f"min_cluster_size: {min_partition_size}",
            f"max_clustering_iterations: {training_iterations}",
            "single_machine_center_initialization: "
            + ("RANDOM_INITIALIZATION" if random_init else "DEFAULT_KMEANS_PLUS_PLUS"),
            'partitioning_distance { distance_measure: "SquaredL2Distance" }',
            f"query_spilling {{ spilling_type: FIXED_NUMBER_OF_CENTERS "
            f"max_spill_centers: {num_leaves_to_search} }}",
            f"expected_sample_size: {training_sample_size}",
            f"query_tokenization_distance_override {distance_measure}",
            f"partitioning_type: {'SPHERICAL' if spherical else 'GENERIC'}",
            f"query_tokenization_type: {'FIXED_POINT_INT8' if quantize_centroids else 'FLOAT'}",
        ]
        if isinstance(incremental_threshold, int):
            lines.append(f"incremental_training_config {{ number_of_datapoints: "
                         f"{incremental_threshold} }}")
        elif isinstance(incremental_threshold, float):
            lines.append(f"incremental_training_config {{ fraction: {incremental_threshold} }}")
        if avq is not None:
            if self.distance_measure != "dot_product":
                raise ValueError("AVQ only applies to dot product distance.")
            lines.append(f"avq: {avq}")
        if soar_lambda is not None:
            if self.distance_measure != "dot_product":
                raise ValueError("SOAR requires dot product distance.")
            extra = (f" overretrieve_factor: {overretrieve_factor}"
                     if overretrieve_factor is not None else "")
            lines.append("database_spilling { spilling_type: TWO_CENTER_ORTHOGONALITY_AMPLIFIED"
                         f" orthogonality_amplification_lambda: {soar_lambda}{extra} }}")
        if projection:
            lines.append(projection)
        if upper_tree is not None:
            lines.append(f"bottom_up_top_level_partitioner {{ {upper_tree} }}")
        return "partitioning {\n" + "\n".join(lines) + "\n}"

    # -- scoring --------------------------------------------------------------
    @_stanza("score_ah")
    def score_ah(self, dimensions_per_block, anisotropic_quantization_threshold=float("nan"),
                 training_sample_size=100000, min_cluster_size=100, hash_type="lut16",
                 training_iterations=10, residual_quantization=None, n_dims=None,
                 projection=None):
        del min_cluster_size  # deprecated in the reference too
        kinds = {"lut16": (16, "INT8_LUT16"), "lut256": (256, "INT8")}
        if hash_type not in kinds:
            raise ValueError(f"hash_type must be one of {list(kinds)}")
        clusters, lookup = kinds[hash_type]
        full, partial = divmod(n_dims, dimensions_per_block)
        if projection is not None:
            proj = f"projection_type: CHUNK num_dims_per_block: {dimensions_per_block}"
        elif partial == 0:
            proj = (f"input_dim: {n_dims} projection_type: CHUNK num_blocks: {full} "
                    f"num_dims_per_block: {dimensions_per_block}")
        else:
            proj = (f"input_dim: {n_dims} projection_type: VARIABLE_CHUNK "
                    f"variable_blocks {{ num_blocks: {full} num_dims_per_block: "
                    f"{dimensions_per_block} }} variable_blocks {{ num_blocks: 1 "
                    f"num_dims_per_block: {partial} }}")
        # global top-N: LUT16 + int16 accumulation (<= 256 blocks) + residuals
        num_blocks = full + (1 if partial else 0)
        global_topn = hash_type == "lut16" and num_blocks <= 256 and bool(residual_quantization)
        return "\n".join([
            "hash {", "asymmetric_hash {",
            f"lookup_type: {lookup}",
            f"use_residual_quantization: {_b(residual_quantization)}",
            f"use_global_topn: {_b(global_topn)}",
            'quantization_distance { distance_measure: "SquaredL2Distance" }',
            f"num_clusters_per_block: {clusters}",
            f"projection {{ {proj} }}",
            "fixed_point_lut_conversion_options { float_to_int_conversion_method: ROUND }",
            f"noise_shaping_threshold: {anisotropic_quantization_threshold}",
            f"expected_sample_size: {training_sample_size}",
            f"max_clustering_iterations: {training_iterations}",
            "}", "}"])

    @_stanza("score_bf")
    def score_brute_force(self, quantize=ReorderType.FLOAT32):
        q = _as_reorder_type(quantize)
        kind = "bfloat16" if q == ReorderType.BFLOAT16 else "fixed_point"
        return f"brute_force {{ {kind} {{ enabled: {q != ReorderType.FLOAT32} }} }}"

    @_stanza("reorder")
    def reorder(self, reordering_num_neighbors, quantize=ReorderType.FLOAT32,
                anisotropic_quantization_threshold=float("nan")):
        q = _as_reorder_type(quantize)
        kind = "bfloat16" if q == ReorderType.BFLOAT16 else "fixed_point"
        return (f"exact_reordering {{ approx_num_neighbors: {reordering_num_neighbors} "
                f"{kind} {{ enabled: {q != ReorderType.FLOAT32} noise_shaping_threshold: "
                f"{anisotropic_quantization_threshold} }} }}")

    @_stanza("autopilot")
    def autopilot(self, mode=IncrementalMode.NONE, quantize=ReorderType.FLOAT32):
        return (f"autopilot {{ tree_ah {{ incremental_mode: {mode.name} "
                f"reordering_dtype: {_as_reorder_type(quantize).name} }} }}")

    # -- assembly ---------------------------------------------------------------
    def create_config(self):
        measures = {"dot_product": '{distance_measure: "DotProductDistance"}',
                    "squared_l2": '{distance_measure: "SquaredL2Distance"}'}
        if self.distance_measure not in measures:
            raise ValueError(f"distance_measure must be one of {list(measures)}")
        dm = measures[self.distance_measure]
        parts = [f"num_neighbors: {self.num_neighbors}", f"distance_measure {dm}"]
        p = self.params
        if "autopilot" in p:
            parts.append(self.autopilot.proto_maker(self, **p["autopilot"]))
            return "\n".join(parts)
        if "pca" in p and "truncate" in p:
            raise ValueError("Exactly 1 of pca or truncate must be set")
        projection = None
        if "pca" in p:
            projection = self.pca.proto_maker(self, **p["pca"])
        elif "truncate" in p:
            projection = self.truncate.proto_maker(self, **p["truncate"])
        tree = p.get("tree")
        if tree is not None:
            tree["distance_measure"] = dm
            upper = p.get("upper_tree")
            if upper is not None:
                upper = self.upper_tree.proto_maker(self, **upper)
            parts.append(self.tree.proto_maker(self, **tree, projection=projection,
                                               upper_tree=upper))
        ah, bf = p.get("score_ah"), p.get("score_bf")
        if (ah is None) == (bf is None):
            raise ValueError("Exactly 1 of score_ah or score_brute_force must be set")
        if ah is not None:
            if "residual_quantization" not in ah:
                ah["residual_quantization"] = (tree is not None
                                               and self.distance_measure == "dot_product")
            ah["n_dims"] = self.db.shape[1]
            parts.append(self.score_ah.proto_maker(self, **ah, projection=projection))
        else:
            parts.append(self.score_brute_force.proto_maker(self, **bf))
        if "reorder" in p:
            parts.append(self.reorder.proto_maker(self, **p["reorder"]))
        return "\n".join(parts)

    def build(self, docids=None, **kwargs):
        if self.builder_lambda is None:
            raise Exception("build() called but no builder lambda was set.")
        return self.builder_lambda(self.db, self.create_config(), self.training_threads,
                                   docids=docids, **kwargs)


__all__ = ["ScannBuilder", "ReorderType", "IncrementalMode"]
