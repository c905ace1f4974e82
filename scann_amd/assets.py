"""Searcher assets in the reference's on-disk layout.

``ScannInterface::Serialize`` (scann/scann_ops/cc/scann.cc:504-601) writes an
artifacts directory that ``load_searcher`` reads back
(scann/scann_ops/py/scann_ops_pybind.py:250-270, scann.cc:105-264):

=========================  ==============================================
scann_config.pb            binary ``ScannConfig`` (io_oss_wrapper.cc:55-77)
scann_assets.pbtxt         text ``ScannAssets`` (scann_npy.cc:272-282)
ah_codebook.pb             binary ``CentersForAllSubspaces``
                           (asymmetric_hashing2/training_model.cc:104-126)
serialized_partitioner.pb  binary ``SerializedPartitioner``
                           (kmeans_tree_partitioner.cc:443-454)
datapoint_to_token.npy     int32 [N], or [2N] with SOAR (-1 = no 2nd leaf)
hashed_dataset.npy         uint8 [N][num_blocks], one 4-bit code per byte
hashed_dataset_soar.npy    uint8 [N][num_blocks], codes in the 2nd leaf
dataset.npy                float32 [N][dim], for the exact reorder
=========================  ==============================================

This module reads and writes that layout for the tree-AH LUT16 searcher, so
an artifacts directory moves between the reference and this build in either
direction.  There is no protobuf runtime in this image: the wire format is
decoded and encoded here, against a schema table holding the subset of the
reference's .proto fields the tree-AH path's configs use
(scann/proto/{scann,partitioning,hash,projection,exact_reordering,
brute_force,distance_measure,input_output,centers}.proto,
scann/trees/kmeans_tree/kmeans_tree.proto,
scann/partitioning/{partitioner,kmeans_tree_partitioner}.proto,
scann/data_format/features.proto, scann/scann_ops/scann_assets.proto).
Unknown fields in a binary file are skipped (as protobuf keeps-and-ignores
them); a config field this schema does not know cannot be written and
raises ValueError.

The pickled ``scann_docids.pkl`` the reference's Python wrapper writes is
never read here (loading it would execute code from the file); docids travel
as JSON (scann_ops_pybind.py).

Parity: the layout and field numbers follow the reference sources cited
above; no reference-written artifacts directory exists in this container, so
byte-level agreement with files produced by the reference binary is
unpinned.  Round trips (write -> read -> identical index and search results)
are tested in tests/test_assets.py.
"""
from __future__ import annotations

import os
import struct
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from .config import SearchConfig, parse_text_proto, search_config_from_tree
from .index import METRIC_NAMES, TreeAHIndex

# --------------------------------------------------------------------------
# protobuf wire format
# --------------------------------------------------------------------------
_VARINT, _I64, _LEN, _I32 = 0, 1, 2, 5


def _read_varint(buf: bytes, pos: int) -> Tuple[int, int]:
    result = shift = 0
    while True:
        if pos >= len(buf):
            raise ValueError("truncated varint")
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7
        if shift >= 70:
            raise ValueError("varint too long")


def wire_fields(buf: bytes):
    """Yield (field_number, wire_type, value) over one serialized message.
    value: int for varints, raw 4/8 bytes for fixed, bytes for LEN."""
    pos, n = 0, len(buf)
    while pos < n:
        key, pos = _read_varint(buf, pos)
        num, wt = key >> 3, key & 7
        if num == 0:
            raise ValueError("field number 0 in protobuf message")
        if wt == _VARINT:
            val, pos = _read_varint(buf, pos)
        elif wt == _I64:
            val, pos = buf[pos:pos + 8], pos + 8
        elif wt == _I32:
            val, pos = buf[pos:pos + 4], pos + 4
        elif wt == _LEN:
            ln, pos = _read_varint(buf, pos)
            val, pos = buf[pos:pos + ln], pos + ln
        else:
            raise ValueError(f"unsupported wire type {wt}")
        if pos > n:
            raise ValueError("truncated protobuf message")
        yield num, wt, val


def _enc_varint(v: int) -> bytes:
    if v < 0:
        v += 1 << 64          # int32/int64 negatives: ten-byte two's complement
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(num: int, wt: int) -> bytes:
    return _enc_varint((num << 3) | wt)


def _enc_len(num: int, payload: bytes) -> bytes:
    return _key(num, _LEN) + _enc_varint(len(payload)) + payload


def _signed(v: int, bits: int) -> int:
    v &= (1 << bits) - 1
    return v - (1 << bits) if v >> (bits - 1) else v


def _packed(wt: int, val, fmt: str) -> np.ndarray:
    """A repeated float/double field, packed (LEN) or one element (fixed)."""
    dt = np.dtype("<" + fmt)
    return np.frombuffer(bytes(val), dtype=dt)


# --------------------------------------------------------------------------
# schema: field number -> (name, kind, sub); kind is a scalar type name,
# "enum" (sub = {name: number}) or "msg" (sub = schema name)
# --------------------------------------------------------------------------
def _enum(*names_and_numbers) -> Dict[str, int]:
    return dict(names_and_numbers)


_DMC = {1: ("distance_measure", "string", None)}
_SCHEMA: Dict[str, Dict[int, Tuple[str, str, Any]]] = {
    "DistanceMeasureConfig": _DMC,
    "ScannConfig": {
        32: ("dataset_name", "string", None),
        3: ("num_neighbors", "int32", None),
        4: ("epsilon_distance", "float", None),
        5: ("distance_measure", "msg", "DistanceMeasureConfig"),
        17: ("exact_reordering", "msg", "ExactReordering"),
        6: ("input_output", "msg", "InputOutputConfig"),
        7: ("brute_force", "msg", "BruteForceConfig"),
        8: ("partitioning", "msg", "PartitioningConfig"),
        13: ("hash", "msg", "HashConfig"),
        21: ("num_single_shard_neighbors", "int32", None),
    },
    "InputOutputConfig": {
        2: ("in_memory_data_type", "enum", _enum(("INT8", 0), ("UINT8", 1), ("INT16", 2),
                                                  ("INT32", 4), ("UINT32", 5), ("INT64", 6),
                                                  ("FLOAT", 8), ("DOUBLE", 9),
                                                  ("IN_MEMORY_DATA_TYPE_NOT_SPECIFIED", 255))),
        5: ("norm_type", "enum", _enum(("NONE", 0), ("UNITL2NORM", 1), ("STDGAUSSNORM", 2),
                                        ("UNITL1NORM", 3))),
        6: ("non_negative", "bool", None),
        7: ("is_dense", "bool", None),
        21: ("pure_dynamic_config", "msg", "PureDynamicConfig"),
    },
    "PureDynamicConfig": {
        1: ("num_shards", "int32", None),
        2: ("vector_type", "enum", _enum(("UNSPECIFIED_VECTOR_TYPE", 0), ("SPARSE", 1),
                                          ("DENSE", 2))),
        3: ("dimensionality", "uint64", None),
    },
    "FixedPoint": {
        1: ("enabled", "bool", None),
        2: ("fixed_point_multiplier", "float", None),
        6: ("fixed_point_multiplier_quantile", "float", None),
        8: ("noise_shaping_threshold", "double", None),
    },
    "Bfloat16": {
        1: ("enabled", "bool", None),
        2: ("noise_shaping_threshold", "double", None),
    },
    "ExactReordering": {
        1: ("approx_num_neighbors", "int32", None),
        2: ("approx_epsilon_distance", "float", None),
        3: ("approx_distance_measure", "msg", "DistanceMeasureConfig"),
        4: ("use_fixed_point_if_possible", "bool", None),
        5: ("fixed_point", "msg", "FixedPoint"),
        7: ("bfloat16", "msg", "Bfloat16"),
    },
    "BruteForceConfig": {
        1: ("scalar_quantized", "bool", None),
        4: ("fixed_point", "msg", "FixedPoint"),
        5: ("bfloat16", "msg", "Bfloat16"),
    },
    "IncrementalTrainingConfig": {
        1: ("fraction", "float", None),
        2: ("number_of_datapoints", "uint32", None),
        3: ("cluster_stability_size", "uint32", None),
        4: ("autopilot", "bool", None),
    },
    "DatabaseSpillingConfig": {
        1: ("spilling_type", "enum", _enum(("NO_SPILLING", 0), ("MULTIPLICATIVE", 1),
                                            ("ADDITIVE", 2), ("FIXED_NUMBER_OF_CENTERS", 3),
                                            ("TWO_CENTER_ORTHOGONALITY_AMPLIFIED", 4),
                                            ("SOAR", 4))),
        2: ("replication_factor", "float", None),
        3: ("max_spill_centers", "uint32", None),
        4: ("orthogonality_amplification_lambda", "float", None),
        5: ("overretrieve_factor", "float", None),
    },
    "QuerySpillingConfig": {
        1: ("spilling_type", "enum", _enum(("NO_SPILLING", 0), ("MULTIPLICATIVE", 1),
                                            ("ADDITIVE", 2), ("ABSOLUTE_DISTANCE", 3),
                                            ("FIXED_NUMBER_OF_CENTERS", 4))),
        2: ("spilling_threshold", "float", None),
        3: ("max_spill_centers", "uint32", None),
    },
    "PartitioningConfig": {
        1: ("num_partitioning_epochs", "int32", None),
        3: ("num_children", "int32", None),
        4: ("partitioning_sampling_fraction", "float", None),
        6: ("max_clustering_iterations", "int32", None),
        7: ("clustering_convergence_tolerance", "float", None),
        8: ("partitioner_prefix", "string", None),
        9: ("min_cluster_size", "float", None),
        10: ("partitioning_distance", "msg", "DistanceMeasureConfig"),
        20: ("database_spilling", "msg", "DatabaseSpillingConfig"),
        21: ("query_spilling", "msg", "QuerySpillingConfig"),
        23: ("partitioning_type", "enum", _enum(("GENERIC", 0), ("SPHERICAL", 1))),
        24: ("database_tokenization_distance_override", "msg", "DistanceMeasureConfig"),
        25: ("query_tokenization_distance_override", "msg", "DistanceMeasureConfig"),
        27: ("clustering_seed", "int32", None),
        28: ("query_tokenization_type", "enum", _enum(("FLOAT", 1), ("FIXED_POINT_INT8", 2),
                                                      ("ASYMMETRIC", 3))),
        29: ("database_tokenization_type", "enum", _enum(("FLOAT", 1), ("FIXED_POINT_INT8", 2),
                                                         ("ASYMMETRIC", 3))),
        31: ("tree_type", "enum", _enum(("KMEANS_TREE", 0), ("PCA_TREE", 1),
                                         ("RANDOM_PROJECTION_TREE", 2), ("BALL_TREE", 3),
                                         ("RANDOM", 4), ("TREE_X_HYBRID", 5))),
        34: ("desired_average_cluster_size", "int32", None),
        35: ("balancing_type", "enum", _enum(("DEFAULT_UNBALANCED", 0), ("GREEDY_BALANCED", 1),
                                              ("UNBALANCED_FLOAT32", 2))),
        38: ("num_mini_batches", "int32", None),
        40: ("max_cluster_size", "int32", None),
        41: ("perturbation", "double", None),
        45: ("expected_sample_size", "int32", None),
        49: ("single_machine_center_initialization", "enum",
             _enum(("DEFAULT_KMEANS_PLUS_PLUS", 0), ("RANDOM_INITIALIZATION", 1))),
        51: ("avq", "float", None),
        52: ("incremental_training_config", "msg", "IncrementalTrainingConfig"),
        53: ("num_tokenized_branch", "int32", None),
        55: ("ignore_empty_cluster_errors", "bool", None),
    },
    "VariableBlock": {
        1: ("num_blocks", "int32", None),
        2: ("num_dims_per_block", "int32", None),
    },
    "ProjectionConfig": {
        1: ("projection_type", "enum", _enum(("NONE", 0), ("CHUNK", 1), ("VARIABLE_CHUNK", 2),
                                              ("RANDOM_GAUSS", 3), ("RANDOM_BINARY", 4),
                                              ("RANDOM_BINARY_DYNAMIC", 5),
                                              ("RANDOM_SPARSE_BINARY", 6),
                                              ("RANDOM_ORTHOGONAL", 7), ("PCA", 8),
                                              ("RANDOM_BILINEAR", 9), ("MEANSTD_PROJECTION", 12),
                                              ("IDENTITY_CHUNK", 13), ("TRUNCATE", 14),
                                              ("EIGENVALUE_OPQ", 15))),
        2: ("num_blocks", "int32", None),
        3: ("num_dims_per_block", "int32", None),
        4: ("variable_blocks", "msg", "VariableBlock"),
        5: ("seed", "int32", None),
        6: ("is_bit_packed", "bool", None),
        7: ("is_dense", "bool", None),
        8: ("build_covariance", "bool", None),
        9: ("input_dim", "uint64", None),
        13: ("pca_significance_threshold", "float", None),
        14: ("pca_truncation_threshold", "float", None),
        15: ("pca_random_rotate_projection_matrix", "bool", None),
    },
    "FixedPointLUTConversionOptions": {
        1: ("float_to_int_conversion_method", "enum", _enum(("TRUNCATE", 0), ("ROUND", 1))),
        2: ("multiplier_quantile", "float", None),
    },
    "AsymmetricHasherConfig": {
        1: ("projection", "msg", "ProjectionConfig"),
        2: ("num_clusters_per_block", "int32", None),
        3: ("max_sample_size", "int32", None),
        4: ("max_clustering_iterations", "int32", None),
        5: ("clustering_convergence_tolerance", "float", None),
        9: ("clustering_seed", "int32", None),
        10: ("sampling_fraction", "float", None),
        11: ("sampling_seed", "int32", None),
        18: ("quantization_distance", "msg", "DistanceMeasureConfig"),
        20: ("lookup_type", "enum", _enum(("FLOAT", 0), ("INT8", 1), ("INT16", 2),
                                           ("INT8_LUT16", 3))),
        22: ("use_residual_quantization", "bool", None),
        23: ("quantization_scheme", "enum", _enum(("PRODUCT", 0), ("STACKED", 1),
                                                   ("PRODUCT_AND_BIAS", 2),
                                                   ("PRODUCT_AND_PACK", 3))),
        25: ("fixed_point_lut_conversion_options", "msg", "FixedPointLUTConversionOptions"),
        28: ("noise_shaping_threshold", "double", None),
        29: ("expected_sample_size", "int32", None),
        31: ("use_norm_biasing_correction", "bool", None),
        32: ("use_normalized_residual_quantization", "bool", None),
        33: ("use_global_topn", "bool", None),
    },
    "HashConfig": {
        1: ("num_bits", "int32", None),
        2: ("projection", "msg", "ProjectionConfig"),
        5: ("asymmetric_hash", "msg", "AsymmetricHasherConfig"),
    },
    "ScannAssets": {
        1: ("assets", "msg", "ScannAsset"),
        2: ("trained_on_the_fly", "bool", None),
    },
    "ScannAsset": {
        1: ("asset_type", "enum", _enum(("UNSPECIFIED_TYPE", 0), ("DATASET", 1),
                                         ("INT8_DATASET", 2), ("AH_DATASET", 3),
                                         ("TOKENIZATION", 4),
                                         ("REORDERING_INT8_MULTIPLIERS", 5),
                                         ("BRUTE_FORCE_INT8_MULTIPLIERS", 6),
                                         ("AH_CENTERS", 7), ("PARTITIONER", 8),
                                         ("DATASET_NPY", 9), ("INT8_DATASET_NPY", 10),
                                         ("AH_DATASET_NPY", 11), ("TOKENIZATION_NPY", 12),
                                         ("INT8_MULTIPLIERS_NPY", 13), ("INT8_NORMS_NPY", 14),
                                         ("BF16_DATASET_NPY", 15),
                                         ("AH_DATASET_SOAR_NPY", 16))),
        2: ("asset_path", "string", None),
    },
}
_BY_NAME = {m: {f[0]: (num,) + f[1:] for num, f in s.items()} for m, s in _SCHEMA.items()}


def _decode_scalar(kind: str, wt: int, val, sub):
    if kind in ("int32", "int64"):
        return _signed(val, 64)        # negatives are sign-extended to 64 bits
    if kind in ("uint32", "uint64"):
        return int(val)
    if kind == "bool":
        return bool(val)
    if kind == "float":
        return float(struct.unpack("<f", val)[0])
    if kind == "double":
        return float(struct.unpack("<d", val)[0])
    if kind == "string":
        return bytes(val).decode("utf-8")
    if kind == "enum":
        num = _signed(val, 64)
        for name, n in sub.items():
            if n == num:
                return name      # first declared name for aliased numbers
        return num
    raise ValueError(kind)


_WIRE = {"int32": _VARINT, "int64": _VARINT, "uint32": _VARINT, "uint64": _VARINT,
         "bool": _VARINT, "enum": _VARINT, "float": _I32, "double": _I64,
         "string": _LEN, "msg": _LEN}


def decode_message(buf: bytes, schema: str) -> Dict[str, List[Any]]:
    """Binary message -> the {field: [values]} tree parse_text_proto builds."""
    fields = _SCHEMA[schema]
    out: Dict[str, List[Any]] = {}
    for num, wt, val in wire_fields(buf):
        if num not in fields:
            continue
        name, kind, sub = fields[num]
        if kind == "msg":
            if wt != _LEN:
                raise ValueError(f"{schema}.{name}: wrong wire type {wt}")
            v = decode_message(val, sub)
        elif wt == _LEN and kind != "string":
            raise ValueError(f"{schema}.{name}: packed encoding of a singular field")
        else:
            if wt != _WIRE[kind]:
                raise ValueError(f"{schema}.{name}: wrong wire type {wt}")
            v = _decode_scalar(kind, wt, val, sub)
        out.setdefault(name, []).append(v)
    return out


def encode_message(tree: Dict[str, List[Any]], schema: str) -> bytes:
    """The inverse of decode_message; fields go out in field-number order as
    protobuf's serializer writes them."""
    names = _BY_NAME[schema]
    parts = []
    for name in tree:
        if name not in names:
            raise ValueError(f"field {name!r} of {schema} is not known to the asset writer")
    for name, values in sorted(tree.items(), key=lambda kv: names[kv[0]][0]):
        num, kind, sub = names[name]
        for v in values:
            if kind == "msg":
                if not isinstance(v, dict):
                    raise ValueError(f"{schema}.{name} must be a message")
                parts.append(_enc_len(num, encode_message(v, sub)))
            elif kind == "string":
                parts.append(_enc_len(num, str(v).encode("utf-8")))
            elif kind == "float":
                parts.append(_key(num, _I32) + struct.pack("<f", float(v)))
            elif kind == "double":
                parts.append(_key(num, _I64) + struct.pack("<d", float(v)))
            elif kind == "enum":
                if isinstance(v, str):
                    if v not in sub:
                        raise ValueError(f"{schema}.{name}: unknown enum value {v!r}")
                    v = sub[v]
                parts.append(_key(num, _VARINT) + _enc_varint(int(v)))
            elif kind == "bool":
                parts.append(_key(num, _VARINT) + _enc_varint(1 if v else 0))
            else:
                if isinstance(v, bool) or not isinstance(v, int):
                    if isinstance(v, float) and v.is_integer():
                        v = int(v)
                    else:
                        raise ValueError(f"{schema}.{name}: integer expected, got {v!r}")
                parts.append(_key(num, _VARINT) + _enc_varint(int(v)))
    return b"".join(parts)


# --------------------------------------------------------------------------
# payload messages (read/written directly, no tree)
# --------------------------------------------------------------------------
def _gfv_values(buf: bytes) -> np.ndarray:
    """GenericFeatureVector (features.proto) dense values: feature_value_float
    (4), feature_value_double (5) or feature_value_int64 (3)."""
    chunks = []
    for num, wt, val in wire_fields(buf):
        if num == 4:
            chunks.append(_packed(wt, val, "f4").astype(np.float64))
        elif num == 5:
            chunks.append(_packed(wt, val, "f8"))
        elif num == 3:
            if wt == _LEN:
                ints, p = [], 0
                while p < len(val):
                    x, p = _read_varint(val, p)
                    ints.append(_signed(x, 64))
            else:
                ints = [_signed(val, 64)]
            chunks.append(np.asarray(ints, np.float64))
        elif num == 6:
            raise ValueError("sparse GenericFeatureVector in an AH codebook")
    return np.concatenate(chunks) if chunks else np.zeros(0)


def read_ah_codebook(buf: bytes) -> Tuple[List[np.ndarray], int]:
    """CentersForAllSubspaces (centers.proto) -> per block [centers][dims]
    float64 arrays and the quantization_scheme."""
    blocks, scheme = [], 0
    for num, wt, val in wire_fields(buf):
        if num == 1:
            centers = [_gfv_values(v) for n, w, v in wire_fields(val) if n == 1]
            if not centers or len({len(c) for c in centers}) != 1:
                raise ValueError("AH codebook block with ragged or no centers")
            blocks.append(np.stack(centers))
        elif num == 2:
            scheme = int(val)
        elif num == 3:
            raise ValueError("AH codebook with a serialized projection is not supported")
    if not blocks:
        raise ValueError("AH codebook has no blocks")
    return blocks, scheme


def write_ah_codebook(codebook: np.ndarray, dim: int) -> bytes:
    """Model::ToProto (training_model.cc:104-126): one GFV of doubles per
    center, the last block trimmed to the dims it covers."""
    B, C, dpb = codebook.shape
    out = []
    for b in range(B):
        width = min(dpb, dim - b * dpb)
        centers = b"".join(
            _enc_len(1, _key(1, _VARINT) + _enc_varint(3)  # feature_type DOUBLE
                     + _enc_len(5, np.ascontiguousarray(codebook[b, c, :width], "<f8").tobytes()))
            for c in range(C))
        out.append(_enc_len(1, centers))
    out.append(_key(2, _VARINT) + _enc_varint(0))          # quantization_scheme PRODUCT
    return b"".join(out)


def _kmeans_node(buf: bytes) -> dict:
    """SerializedKMeansTree.Node (kmeans_tree.proto); a center's
    float_dimension wins over its double dimension when present
    (KMeansTreeNode::BuildFromProto, kmeans_tree_node.cc:91-124)."""
    node = {"centers": [], "children": [], "leaf_id": -1}
    for num, wt, val in wire_fields(buf):
        if num == 1:
            dbl, flt = [], []
            for n, w, v in wire_fields(val):
                if n == 1:
                    dbl.append(_packed(w, v, "f8"))
                elif n == 2:
                    flt.append(_packed(w, v, "f4"))
            vals = np.concatenate(flt) if flt and sum(map(len, flt)) else \
                (np.concatenate(dbl) if dbl else np.zeros(0))
            node["centers"].append(vals.astype(np.float32))
        elif num == 3:
            node["children"].append(_kmeans_node(val))
        elif num == 5:
            node["leaf_id"] = _signed(val, 64)
    return node


def read_partitioner(buf: bytes) -> np.ndarray:
    """SerializedPartitioner (partitioner.proto) of a one-level k-means tree
    -> leaf centers [n_tokens][dim] float32, row = token (leaf_id)."""
    n_tokens, kmeans = None, None
    for num, wt, val in wire_fields(buf):
        if num == 1:
            n_tokens = _signed(val, 64)
        elif num == 2:
            kmeans = val
        elif num == 3 and val:
            raise ValueError("projected partitioners are not supported")
        elif num == 4:
            raise ValueError("linear-projection-tree partitioners are not supported")
    if kmeans is None:
        raise ValueError("serialized partitioner has no k-means tree")
    tree = None
    for num, wt, val in wire_fields(kmeans):
        if num == 1:
            tree = val
        elif num == 6:
            raise ValueError("bottom-up multi-level partitioners are not supported")
    if tree is None:
        raise ValueError("serialized partitioner has no k-means tree")
    root = None
    for num, wt, val in wire_fields(tree):
        if num == 1:
            root = _kmeans_node(val)
    if root is None or not root["children"]:
        raise ValueError("k-means tree has no leaves")
    kids = root["children"]
    if len(root["centers"]) != len(kids):
        raise ValueError("k-means tree root: centers and children differ in number")
    if any(k["children"] for k in kids):
        raise ValueError("multi-level k-means trees are not supported (one level only)")
    L = len(kids)
    # KMeansTree::NumberLeaves numbers leaves depth first; a tree written
    # without ids falls back to that order.
    ids = [k["leaf_id"] if k["leaf_id"] >= 0 else i for i, k in enumerate(kids)]
    if sorted(ids) != list(range(L)):
        raise ValueError("k-means tree leaf ids are not 0..L-1")
    if n_tokens is not None and n_tokens != L:
        raise ValueError(f"n_tokens {n_tokens} != {L} leaves")
    dims = {len(c) for c in root["centers"]}
    if len(dims) != 1:
        raise ValueError("k-means centers of different dimensionality")
    centers = np.zeros((L, dims.pop()), np.float32)
    for i, t in enumerate(ids):
        centers[t] = root["centers"][i]
    return centers


def write_partitioner(centers: np.ndarray) -> bytes:
    """KMeansTreePartitioner::CopyToProto (kmeans_tree_partitioner.cc:443-454)
    of a one-level tree, written without indices (kmeans_tree.cc:111-115)."""
    L = centers.shape[0]
    node = [_enc_len(1, _enc_len(1, np.ascontiguousarray(c, "<f8").tobytes()))
            for c in np.asarray(centers, np.float64)]
    for i in range(L):
        leaf = _key(4, _I64) + struct.pack("<d", 0.0) + _key(5, _VARINT) + _enc_varint(i)
        node.append(_enc_len(3, leaf))
    node.append(_key(4, _I64) + struct.pack("<d", 0.0) + _key(5, _VARINT) + _enc_varint(-1))
    tree = _enc_len(1, b"".join(node)) + _key(3, _VARINT) + _enc_varint(0)
    return _key(1, _VARINT) + _enc_varint(L) + _enc_len(2, _enc_len(1, tree))


# --------------------------------------------------------------------------
# artifacts directory
# --------------------------------------------------------------------------
def read_config(path: str) -> Tuple[Dict[str, List[Any]], SearchConfig]:
    with open(path, "rb") as f:
        tree = decode_message(f.read(), "ScannConfig")
    return tree, search_config_from_tree(tree)


def parse_assets(text: str, artifacts_dir: str) -> Dict[str, str]:
    """scann_assets.pbtxt -> {asset_type: path}; relative paths are resolved
    against the artifacts directory (RewriteAssetFilenameIfRelative,
    scann.cc:236-244)."""
    tree = parse_text_proto(text)
    out: Dict[str, str] = {}
    for a in tree.get("assets", []):
        kind = a.get("asset_type", [None])[0]
        path = a.get("asset_path", [None])[0]
        if kind is None or path is None:
            raise ValueError("asset without asset_type or asset_path")
        out[str(kind)] = path if os.path.isabs(path) else os.path.join(artifacts_dir, path)
    return out


def is_reference_layout(assets: Dict[str, str]) -> bool:
    return "AH_CENTERS" in assets or "PARTITIONER" in assets


def _has_soar(cfg_tree) -> bool:
    """HasSoar (scann.cc): database spilling of the two-center kind."""
    part = cfg_tree.get("partitioning", [{}])[0]
    spill = part.get("database_spilling", [{}])[0]
    return spill.get("spilling_type", ["NO_SPILLING"])[0] in (
        "SOAR", "TWO_CENTER_ORTHOGONALITY_AMPLIFIED", 4)


def load_artifacts(artifacts_dir: str, assets_pbtxt: Optional[str] = None
                   ) -> Tuple[TreeAHIndex, Dict[str, List[Any]], SearchConfig]:
    """ScannInterface::LoadArtifacts (scann.cc:105-264) for the tree-AH
    LUT16 searcher -> (TreeAHIndex, config tree, SearchConfig)."""
    tree, cfg = read_config(os.path.join(artifacts_dir, "scann_config.pb"))
    if assets_pbtxt is None:
        with open(os.path.join(artifacts_dir, "scann_assets.pbtxt")) as f:
            assets_pbtxt = f.read()
    assets = parse_assets(assets_pbtxt, artifacts_dir)
    for need in ("AH_CENTERS", "PARTITIONER", "TOKENIZATION_NPY", "AH_DATASET_NPY"):
        if need not in assets:
            raise ValueError(f"tree-AH artifacts need a {need} asset")
    with open(assets["AH_CENTERS"], "rb") as f:
        blocks, scheme = read_ah_codebook(f.read())
    if scheme != 0:
        raise ValueError("only PRODUCT quantization codebooks are supported")
    with open(assets["PARTITIONER"], "rb") as f:
        centers = read_partitioner(f.read())
    L, dim = centers.shape
    B = len(blocks)
    if any(b.shape[0] != 16 for b in blocks):
        raise ValueError("LUT16 needs 16 centers per AH block")
    dpb = blocks[0].shape[1]
    widths = [b.shape[1] for b in blocks]
    if any(w != dpb for w in widths[:-1]) or not 0 < widths[-1] <= dpb or \
            sum(widths) != dim:
        raise ValueError(f"AH blocks of {widths} dims do not chunk dim {dim}")
    codebook = np.zeros((B, 16, dpb), np.float32)
    for b, c in enumerate(blocks):
        codebook[b, :, :c.shape[1]] = c

    tokens = np.load(assets["TOKENIZATION_NPY"], allow_pickle=False)
    hashed = np.load(assets["AH_DATASET_NPY"], allow_pickle=False)
    if tokens.dtype != np.int32 or hashed.dtype != np.uint8 or hashed.ndim != 2:
        raise ValueError("tokenization must be int32 and the hashed dataset 2-D uint8")
    N = hashed.shape[0]
    if hashed.shape[1] != B:
        raise ValueError(f"hashed dataset has {hashed.shape[1]} blocks, codebook {B}")
    soar = _has_soar(tree)
    mult = 2 if soar else 1
    if tokens.shape != (mult * N,):
        raise ValueError(f"datapoint_to_token has shape {tokens.shape}, expected ({mult * N},)")
    if np.any(tokens >= L) or np.any(tokens[::mult] < 0) or np.any(tokens < -1):
        raise ValueError("datapoint_to_token holds tokens outside the partitioner")
    # AddTokenizationToOptions (scann.cc:80-98): entry j goes to leaf
    # tokens[j] as datapoint j // mult, in entry order (ascending per leaf).
    entry = np.flatnonzero(tokens >= 0)
    leaf = tokens[entry].astype(np.int64)
    order = np.argsort(leaf, kind="stable")
    entry, leaf = entry[order], leaf[order]
    dp = (entry // mult).astype(np.int64)
    codes = hashed[dp]
    if soar:
        if "AH_DATASET_SOAR_NPY" not in assets:
            raise ValueError("SOAR artifacts need an AH_DATASET_SOAR_NPY asset")
        soar_codes = np.load(assets["AH_DATASET_SOAR_NPY"], allow_pickle=False)
        if soar_codes.shape != hashed.shape or soar_codes.dtype != np.uint8:
            raise ValueError("SOAR hashed dataset does not match the hashed dataset")
        # tree_ah_hybrid_residual.cc:384-394: the 2nd-token copy's codes
        secondary = tokens[1::2][dp] == leaf
        codes[secondary] = soar_codes[dp[secondary]]
    offsets = np.zeros(L + 1, np.uint64)
    offsets[1:] = np.cumsum(np.bincount(leaf, minlength=L))
    dataset = None
    if "DATASET_NPY" in assets:
        dataset = np.load(assets["DATASET_NPY"], allow_pickle=False)
        if dataset.dtype != np.float32 or dataset.shape != (N, dim):
            raise ValueError("dataset.npy must be float32 [N][dim]")
    elif cfg.has_reordering:
        raise ValueError("config asks for exact reordering but there is no DATASET_NPY asset")
    index = TreeAHIndex(
        metric=METRIC_NAMES[cfg.metric], dim=dim, num_blocks=B, dims_per_block=dpb,
        residual=cfg.residual, centers=centers, codebook=codebook, leaf_offsets=offsets,
        leaf_members=dp.astype(np.uint32), member_codes=codes, num_datapoints=N,
        dataset=dataset if cfg.has_reordering else None,
        spilling_overretrieve_factor=cfg.overretrieve_factor if soar else 1.0)
    return index, tree, cfg


def save_artifacts(index: TreeAHIndex, config_text: str, path: str,
                   relative_path: bool = False) -> str:
    """ScannInterface::Serialize (scann.cc:504-601) + ScannNumpy::Serialize
    (scann_npy.cc:272-282) for a whole tree-AH index; returns the assets
    text it wrote to scann_assets.pbtxt."""
    if index.is_shard:
        raise ValueError("serialize the whole index, not a shard")
    tree = parse_text_proto(config_text)
    cfg = search_config_from_tree(tree)
    os.makedirs(path, exist_ok=True)
    assets: List[Tuple[str, str]] = []

    def target(name: str, kind: str) -> str:
        full = os.path.join(path, name)
        assets.append((kind, name if relative_path else full))
        return full

    with open(os.path.join(path, "scann_config.pb"), "wb") as f:
        f.write(encode_message(tree, "ScannConfig"))
    with open(target("ah_codebook.pb", "AH_CENTERS"), "wb") as f:
        f.write(write_ah_codebook(index.codebook, index.dim))
    with open(target("serialized_partitioner.pb", "PARTITIONER"), "wb") as f:
        f.write(write_partitioner(index.centers))

    N, B, L = index.num_datapoints, index.num_blocks, index.num_leaves
    leaf = np.repeat(np.arange(L, dtype=np.int32), index.leaf_sizes())
    members = index.leaf_members.astype(np.int64)
    soar = _has_soar(tree)
    hashed = np.zeros((N, B), np.uint8)
    if soar:
        # the 2N layout: a datapoint's lower leaf first, -1 when not spilled;
        # codes of the lower leaf in hashed_dataset, of the higher one in
        # hashed_dataset_soar (CombineLeafDatasets, tree_x_hybrid/internal/utils.h:86-104)
        tokens = np.full(2 * N, -1, np.int32)
        soar_codes = np.zeros((N, B), np.uint8)
        first = np.zeros(N, bool)
        for l_, m, c in zip(leaf, members, index.member_codes):
            if not first[m]:
                first[m] = True
                tokens[2 * m] = l_
                hashed[m] = c
            else:
                if tokens[2 * m + 1] != -1:
                    raise ValueError(f"datapoint {m} is in more than two leaves")
                tokens[2 * m + 1] = l_
                soar_codes[m] = c
    else:
        if index.num_members != N or np.unique(members).size != N:
            raise ValueError("a non-spilled index must hold every datapoint exactly once")
        tokens = np.zeros(N, np.int32)
        tokens[members] = leaf
        hashed[members] = index.member_codes
    if soar and not np.all(tokens[0::2] >= 0):
        raise ValueError("every datapoint needs a leaf")
    np.save(target("datapoint_to_token.npy", "TOKENIZATION_NPY"), tokens)
    np.save(target("hashed_dataset.npy", "AH_DATASET_NPY"), hashed)
    if soar:
        np.save(target("hashed_dataset_soar.npy", "AH_DATASET_SOAR_NPY"), soar_codes)
    if index.dataset is not None and cfg.has_reordering:
        np.save(target("dataset.npy", "DATASET_NPY"), index.dataset)
    text = format_message({"assets": [{"asset_type": [k], "asset_path": [p]}
                                      for k, p in assets]}, "ScannAssets")
    with open(os.path.join(path, "scann_assets.pbtxt"), "w") as f:
        f.write(text)
    return text


def format_message(tree: Dict[str, List[Any]], schema: str, indent: int = 0) -> str:
    """protobuf TextFormat of a tree in field-number order (enums bare,
    strings quoted, floats as their shortest float32 spelling)."""
    names = _BY_NAME[schema]
    pad = "  " * indent
    lines = []
    for name, values in sorted(tree.items(), key=lambda kv: names.get(kv[0], (1 << 30,))[0]):
        if name not in names:
            raise ValueError(f"field {name!r} of {schema} is not known to the asset writer")
        _, kind, sub = names[name]
        for v in values:
            if kind == "msg":
                lines.append(f"{pad}{name} {{\n{format_message(v, sub, indent + 1)}{pad}}}\n")
                continue
            if kind == "string":
                txt = '"' + str(v).replace("\\", "\\\\").replace('"', '\\"') + '"'
            elif kind == "bool":
                txt = "true" if v else "false"
            elif kind == "float":
                txt = str(np.float32(v))
            elif kind == "double":
                txt = repr(float(v))
            else:
                txt = str(v)
            lines.append(f"{pad}{name}: {txt}\n")
    return "".join(lines)


def config_text(tree: Dict[str, List[Any]]) -> str:
    """TextFormat::PrintToString of a decoded config (ScannNumpy::Config,
    scann_npy.cc:203-208)."""
    return format_message(tree, "ScannConfig")
