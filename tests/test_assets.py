"""Reference-layout artifacts (scann_amd.assets): the
protobuf wire codec against hand-computed bytes from the protobuf encoding
rules, every golden builder config through binary and back, and
save -> load round trips of built indexes (plain, SOAR-spilled, ragged last
AH block).  Bytes written by the reference binary itself are not available
here, so agreement with them is unpinned (see scann_amd/assets.py)."""
import json
import os
import struct

import numpy as np
import pytest

from scann_amd import assets
from scann_amd.config import parse_text_proto, search_config_from_text, search_config_from_tree
from scann_amd.index import METRIC_DOT, METRIC_SQUARED_L2
from scann_amd.index_builder import build_tree_ah

HERE = os.path.dirname(__file__)


def _golden_configs():
    with open(os.path.join(HERE, "golden", "builder_configs.json")) as f:
        return [(c["name"], c["config"]) for c in json.load(f)]


def test_wire_bytes_of_known_fields():
    # key = field << 3 | wire type; num_neighbors (3) varint 10 -> 18 0a
    tree = {"num_neighbors": [10],
            "distance_measure": [{"distance_measure": ["DotProductDistance"]}]}
    got = assets.encode_message(tree, "ScannConfig")
    want = bytes([0x18, 0x0A, 0x2A, 20, 0x0A, 18]) + b"DotProductDistance"
    assert got == want
    assert assets.decode_message(got, "ScannConfig") == tree
    # 300 -> ac 02 ; negative int32 -> ten bytes ; float fixed32 ; enum varint
    t2 = {"num_children": [300], "clustering_seed": [-1], "min_cluster_size": [1.5],
          "partitioning_type": ["SPHERICAL"]}
    b2 = assets.encode_message(t2, "PartitioningConfig")
    assert b2 == (bytes([0x18, 0xAC, 0x02]) + bytes([0x4D]) + struct.pack("<f", 1.5)
                  + bytes([0xB8, 0x01, 0x01])
                  + bytes([0xD8, 0x01]) + b"\xff" * 9 + b"\x01")
    assert assets.decode_message(b2, "PartitioningConfig") == t2


def test_unknown_fields_skipped_on_read_and_refused_on_write():
    blob = assets.encode_message({"num_neighbors": [3]}, "ScannConfig")
    # field 99 (varint) and field 98 (LEN) are not in the schema
    extra = bytes([0x98, 0x06, 0x07, 0x92, 0x06, 0x02, 0x41, 0x42])
    assert assets.decode_message(extra + blob, "ScannConfig") == {"num_neighbors": [3]}
    with pytest.raises(ValueError, match="not known"):
        assets.encode_message({"no_such_field": [1]}, "ScannConfig")
    with pytest.raises(ValueError, match="truncated"):
        list(assets.wire_fields(bytes([0x2A, 0x05, 0x0A])))


def test_spilling_type_alias_reads_back_as_first_name():
    b = assets.encode_message({"spilling_type": ["SOAR"]}, "DatabaseSpillingConfig")
    assert b == bytes([0x08, 0x04])
    assert assets.decode_message(b, "DatabaseSpillingConfig") == {
        "spilling_type": ["TWO_CENTER_ORTHOGONALITY_AMPLIFIED"]}


@pytest.mark.parametrize("name,text", _golden_configs())
def test_golden_configs_survive_binary_and_text(name, text):
    tree = parse_text_proto(text)
    blob = assets.encode_message(tree, "ScannConfig")
    back = assets.decode_message(blob, "ScannConfig")
    assert assets.encode_message(back, "ScannConfig") == blob
    # the printed text parses to the same binary again
    assert assets.encode_message(parse_text_proto(assets.config_text(back)), "ScannConfig") == blob
    try:
        want = search_config_from_text(text)
    except ValueError as e:
        with pytest.raises(ValueError, match=str(e)[:20]):
            search_config_from_tree(back)
        return
    got = search_config_from_tree(back)
    for field in ("num_neighbors", "metric", "num_leaves", "leaves_to_search",
                  "dims_per_block", "residual", "reorder_num_neighbors", "overretrieve_factor"):
        assert getattr(got, field) == getattr(want, field), field
    if want.soar_lambda is not None:
        assert got.soar_lambda == pytest.approx(want.soar_lambda)


def _config(metric: str, leaves: int, blocks: int, dpb: int, dim: int, soar: bool,
            reorder: bool) -> str:
    spill = ("database_spilling { spilling_type: TWO_CENTER_ORTHOGONALITY_AMPLIFIED "
             "orthogonality_amplification_lambda: 1.5 overretrieve_factor: 2.0 }") if soar else ""
    if dim % dpb:
        proj = (f"projection {{ projection_type: VARIABLE_CHUNK input_dim: {dim} "
                f"variable_blocks {{ num_blocks: {blocks - 1} num_dims_per_block: {dpb} }} "
                f"variable_blocks {{ num_blocks: 1 num_dims_per_block: {dim % dpb} }} }}")
    else:
        proj = (f"projection {{ projection_type: CHUNK input_dim: {dim} num_blocks: {blocks} "
                f"num_dims_per_block: {dpb} }}")
    reo = "exact_reordering { approx_num_neighbors: 40 fixed_point { enabled: False } }" \
        if reorder else ""
    residual = "True" if metric == "DotProductDistance" else "False"
    return f"""num_neighbors: 10
distance_measure {{ distance_measure: "{metric}" }}
partitioning {{ num_children: {leaves} max_clustering_iterations: 6
  partitioning_distance {{ distance_measure: "SquaredL2Distance" }}
  query_spilling {{ spilling_type: FIXED_NUMBER_OF_CENTERS max_spill_centers: 4 }}
  {spill} }}
hash {{ asymmetric_hash {{ lookup_type: INT8_LUT16 use_residual_quantization: {residual}
  num_clusters_per_block: 16 {proj} }} }}
{reo}
"""


CASES = [
    # metric, dim, dpb, soar, reorder
    ("DotProductDistance", 32, 2, False, True),
    ("SquaredL2Distance", 24, 4, True, True),
    ("DotProductDistance", 33, 2, True, False),
]


@pytest.mark.parametrize("metric,dim,dpb,soar,reorder", CASES)
@pytest.mark.parametrize("relative", [False, True])
def test_save_load_round_trip(tmp_path, metric, dim, dpb, soar, reorder, relative):
    rng = np.random.default_rng(dim)
    db = rng.standard_normal((1500, dim)).astype(np.float32)
    blocks = -(-dim // dpb)
    m = METRIC_DOT if metric == "DotProductDistance" else METRIC_SQUARED_L2
    ix = build_tree_ah(db, m, 12, dpb, training_iterations=4, ah_training_iterations=3,
                       residual=(m == METRIC_DOT), keep_dataset=reorder,
                       soar_lambda=1.5 if soar else None, seed=3)
    text = _config(metric, 12, blocks, dpb, dim, soar, reorder)
    written = assets.save_artifacts(ix, text, str(tmp_path), relative_path=relative)
    names = sorted(os.listdir(tmp_path))
    want = {"scann_config.pb", "scann_assets.pbtxt", "ah_codebook.pb",
            "serialized_partitioner.pb", "datapoint_to_token.npy", "hashed_dataset.npy"}
    assert want <= set(names)
    assert ("hashed_dataset_soar.npy" in names) == soar
    assert ("dataset.npy" in names) == reorder
    for line in written.splitlines():
        if "asset_path" in line:
            assert os.path.isabs(line.split('"')[1]) != relative

    tokens = np.load(tmp_path / "datapoint_to_token.npy")
    assert tokens.dtype == np.int32 and tokens.shape == ((2 if soar else 1) * 1500,)
    if soar:
        assert np.all(tokens[0::2] >= 0)
        both = tokens[1::2] >= 0
        assert np.all(tokens[0::2][both] < tokens[1::2][both])  # lower leaf first
        assert both.any()

    back, tree, cfg = assets.load_artifacts(str(tmp_path))
    assert cfg.num_leaves == 12 and cfg.has_reordering == reorder
    for f in ("metric", "dim", "num_blocks", "dims_per_block", "num_datapoints"):
        assert getattr(back, f) == getattr(ix, f), f
    assert bool(back.residual) == bool(ix.residual)
    np.testing.assert_array_equal(back.centers, ix.centers)
    np.testing.assert_array_equal(back.codebook, ix.codebook)
    np.testing.assert_array_equal(back.leaf_offsets, ix.leaf_offsets)
    np.testing.assert_array_equal(back.leaf_members, ix.leaf_members)
    np.testing.assert_array_equal(back.member_codes, ix.member_codes)
    if reorder:
        np.testing.assert_array_equal(back.dataset, ix.dataset)
    assert back.disjoint == ix.disjoint
    if soar:
        assert back.spilling_overretrieve_factor == ix.spilling_overretrieve_factor
    # the written assets text is what load_artifacts reads when handed it
    again, _, _ = assets.load_artifacts(str(tmp_path), written)
    np.testing.assert_array_equal(again.member_codes, ix.member_codes)


def test_partitioner_reads_float_centers_and_leaf_ids(tmp_path):
    # hand-built SerializedPartitioner: leaves listed in reverse id order,
    # centers as float_dimension (field 2) as some writers emit them
    c = np.array([[1.0, 2.0], [3.0, 4.0], [5.0, 6.0]], np.float32)
    node = b""
    for row in c[::-1]:
        node += assets._enc_len(1, assets._enc_len(2, row.astype("<f4").tobytes()))
    for leaf in (2, 1, 0):
        node += assets._enc_len(3, assets._key(5, 0) + assets._enc_varint(leaf))
    blob = (assets._key(1, 0) + assets._enc_varint(3)
            + assets._enc_len(2, assets._enc_len(1, assets._enc_len(1, node))))
    np.testing.assert_array_equal(assets.read_partitioner(blob), c)
    # the writer's own bytes read back identically
    np.testing.assert_array_equal(assets.read_partitioner(assets.write_partitioner(c)), c)


def test_partitioner_rejects_multi_level_trees():
    leaf = assets._key(5, 0) + assets._enc_varint(0)
    inner = assets._enc_len(1, assets._enc_len(1, np.zeros(2, "<f8").tobytes())) + \
        assets._enc_len(3, leaf)
    root = assets._enc_len(1, assets._enc_len(1, np.zeros(2, "<f8").tobytes())) + \
        assets._enc_len(3, inner)
    blob = assets._enc_len(2, assets._enc_len(1, assets._enc_len(1, root)))
    with pytest.raises(ValueError, match="one level"):
        assets.read_partitioner(blob)


def test_codebook_gfv_encodings():
    # one block, 16 centers: doubles (field 5), floats (field 4), int64 (3)
    rows = np.arange(32, dtype=np.float64).reshape(16, 2)
    def gfv(field, arr, fmt):
        return assets._enc_len(field, np.ascontiguousarray(arr, fmt).tobytes())
    for field, fmt in ((5, "<f8"), (4, "<f4")):
        blk = b"".join(assets._enc_len(1, gfv(field, r, fmt)) for r in rows)
        blocks, scheme = assets.read_ah_codebook(assets._enc_len(1, blk))
        np.testing.assert_array_equal(blocks[0], rows)
        assert scheme == 0
    ints = b"".join(assets._enc_len(1, assets._enc_len(3, b"".join(
        assets._enc_varint(int(v)) for v in r))) for r in rows)
    np.testing.assert_array_equal(assets.read_ah_codebook(assets._enc_len(1, ints))[0][0], rows)


def test_backcompat_shim_lists_present_assets(tmp_path):
    from scann_amd.scann_ops_pybind import _populate_and_save_assets_proto
    for name in ("ah_codebook.pb", "datapoint_to_token.npy", "dataset.npy"):
        (tmp_path / name).write_bytes(b"")
    _populate_and_save_assets_proto(str(tmp_path))
    listed = assets.parse_assets((tmp_path / "scann_assets.pbtxt").read_text(), str(tmp_path))
    assert set(listed) == {"AH_CENTERS", "TOKENIZATION_NPY", "DATASET_NPY"}
    assert listed["DATASET_NPY"] == str(tmp_path / "dataset.npy")


def test_pickled_docids_are_never_loaded(tmp_path):
    from scann_amd import scann_ops_pybind
    (tmp_path / "scann_assets.pbtxt").write_text("")
    (tmp_path / "scann_docids.pkl").write_bytes(b"\x80\x04N.")
    with pytest.raises(ValueError, match="pickle"):
        scann_ops_pybind.load_searcher(str(tmp_path))


def test_schema_matches_reference_protos():
    """assets.py's field table agrees with the reference's .proto files
    (tests/golden/proto_fields.json, parsed by tests/golden/make_proto_fields.py
    in the build container): every field the codec knows has the reference's
    number and type, every enum value the reference's number."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "proto_fields.json")
    with open(path) as f:
        ref = json.load(f)
    msgs, enums = ref["messages"], ref["enums"]
    bad = []
    for msg, fields in assets._SCHEMA.items():
        pm = msgs.get(msg)
        if pm is None:
            bad.append(("message", msg))
            continue
        for num, (name, kind, sub) in fields.items():
            f = pm.get(name)
            if f is None:
                bad.append(("field", msg, name))
                continue
            if f["number"] != num:
                bad.append(("number", msg, name, num, f["number"]))
            if kind == "msg":
                if f["type"] != sub:
                    bad.append(("message type", msg, name, sub, f["type"]))
            elif kind == "enum":
                en = enums.get(f"{msg}.{f['type']}", enums.get(f["type"]))
                if en is None:
                    bad.append(("enum", msg, name, f["type"]))
                    continue
                for ename, ev in sub.items():
                    if en.get(ename) != ev:
                        bad.append(("enum value", msg, name, ename, ev, en.get(ename)))
            elif f["type"] != kind:
                bad.append(("type", msg, name, kind, f["type"]))
    assert not bad, bad
