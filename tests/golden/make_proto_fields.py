"""Parse the reference's .proto files into tests/golden/proto_fields.json.

    python3 tests/golden/make_proto_fields.py [REFERENCE_ROOT]

Run in the build container (the reference tree is not on the GPU box).  The
fixture holds data only -- per message (nested messages by their simple
name), each field's number, declared type and label; per enum, its value
numbers, nested enums keyed "Message.Enum" -- for the files whose messages
scann_amd/assets.py decodes:
scann.proto and the configs it embeds, scann_assets.proto, centers.proto,
kmeans_tree.proto, partitioner.proto / kmeans_tree_partitioner.proto
(VERDICT r1 item 9).  tests/test_assets.py checks assets.py's schema table
against it.
"""
import json
import os
import re
import sys

FILES = [
    "scann/proto/scann.proto", "scann/proto/input_output.proto",
    "scann/proto/exact_reordering.proto", "scann/proto/brute_force.proto",
    "scann/proto/partitioning.proto", "scann/proto/projection.proto",
    "scann/proto/hash.proto", "scann/proto/distance_measure.proto",
    "scann/proto/centers.proto", "scann/proto/incremental_updates.proto",
    "scann/scann_ops/scann_assets.proto", "scann/trees/kmeans_tree/kmeans_tree.proto",
    "scann/partitioning/partitioner.proto", "scann/partitioning/kmeans_tree_partitioner.proto",
    "scann/partitioning/linear_projection_tree.proto",
]

FIELD = re.compile(r"^(optional|required|repeated)?\s*([A-Za-z_][\w.]*)\s+([A-Za-z_]\w*)\s*=\s*(\d+)")
ENUM_VAL = re.compile(r"^([A-Za-z_]\w*)\s*=\s*(-?\d+)")


def strip_comments(text):
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return "\n".join(line.split("//", 1)[0] for line in text.splitlines())


def statements(text):
    """Split into ';', '{' and '}' terminated statements (declarations may wrap lines)."""
    buf = ""
    for ch in text:
        if ch in "{};":
            yield (buf.strip(), ch)
            buf = ""
        else:
            buf += " " if ch == "\n" else ch
    if buf.strip():
        yield (buf.strip(), "")


def parse(text, messages, enums):
    stack = []   # ("message"|"enum"|"oneof"|"other", name)
    for stmt, term in statements(strip_comments(text)):
        stmt = re.sub(r"\s+", " ", stmt)
        if term == "{":
            m = re.match(r"^(message|enum|oneof|extend|service)\s+([\w.]+)", stmt)
            kind, name = (m.group(1), m.group(2)) if m else ("other", stmt)
            stack.append((kind, name))
            if kind == "message":
                messages.setdefault(name, {})
            elif kind == "enum":
                # a nested enum is keyed by its message: two messages declare
                # different `SpillingType`s
                parent = next((s[1] for s in reversed(stack[:-1]) if s[0] == "message"), None)
                qual = f"{parent}.{name}" if parent else name
                stack[-1] = ("enum", qual)
                enums.setdefault(qual, {})
            continue
        if term == "}":
            if stack:
                stack.pop()
            continue
        if not stack:
            continue
        # innermost message / enum (oneof fields belong to their message)
        owner = next((s for s in reversed(stack) if s[0] in ("message", "enum")), None)
        if owner is None:
            continue
        if owner[0] == "enum" and stack[-1][0] == "enum":
            m = ENUM_VAL.match(stmt)
            if m and not re.match(r"^option\b", stmt):
                enums[owner[1]].setdefault(m.group(1), int(m.group(2)))
            continue
        if owner[0] == "message" and stack[-1][0] in ("message", "oneof"):
            if re.match(r"^(option|reserved|extensions)\b", stmt):
                continue
            m = FIELD.match(stmt)
            if m:
                label, ftype, name, num = m.groups()
                messages[owner[1]][name] = {"number": int(num), "type": ftype.split(".")[-1],
                                            "label": label or "oneof"}


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    messages, enums = {}, {}
    used = []
    for rel in FILES:
        path = os.path.join(root, rel)
        if not os.path.exists(path):
            continue
        used.append(rel)
        with open(path) as f:
            parse(f.read(), messages, enums)
    out = {"source_files": used, "messages": messages, "enums": enums}
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "proto_fields.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(f"{dst}: {len(messages)} messages, {len(enums)} enums from {len(used)} files")


if __name__ == "__main__":
    main()
