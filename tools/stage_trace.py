"""Stage entry points of the glove-shaped index, for per-kernel timing in
isolation (run under rocprofv3 --kernel-trace --stats on the GPU box):

    rocprofv3 --kernel-trace --stats -d out -o run -- python3 tools/stage_trace.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bench import LEAVES_TO_SEARCH, build_index  # noqa: E402
from scann_amd import _native  # noqa: E402


def main():
    db, q, ix = build_index(1_183_514, seed=2)
    nat = _native.NativeIndex(ix)
    for _ in range(10):
        nat.partition_topl(q, LEAVES_TO_SEARCH)
    for _ in range(10):
        nat.create_lookup_tables(q)
    for _ in range(5):
        nat.search_pre_reorder(q, LEAVES_TO_SEARCH, 100)
    print("done", flush=True)


if __name__ == "__main__":
    main()
