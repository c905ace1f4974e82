"""Turn a rocprofv3 --pmc FETCH_SIZE counter collection into
profiles/scan_traffic_<config>.json (bench.py --config <config>).

    python tools/pmc_traffic.py gpurun_out/pmc1/run_counter_collection.csv [config]

FETCH_SIZE is in KiB and, on gfx950, reads exactly half of the bytes of a
wide coalesced streaming read (MI355X_MICROARCH.md, HBM section), so the
per-launch HBM read traffic is 2 * FETCH_SIZE * 1024 bytes.  The file records
the sha256 of smx_kernels.hip's code (comments stripped) so bench.py only
reports it for the same kernel.
"""
import csv
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "lut16_scan_kernel"


def kernel_sha():
    """sha256 of smx_kernels.hip with its comments and blank space removed (a
    comment edit does not make a traffic record stale; any code change does)."""
    sys.path.insert(0, ROOT)
    import bench
    return bench.kernel_source_sha()


def main(path, config="glove"):
    out = os.path.join(ROOT, "profiles", f"scan_traffic_{config}.json")
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if KERNEL in row["Kernel_Name"] and row["Counter_Name"] == "FETCH_SIZE":
                vals.append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit("no FETCH_SIZE rows for the scan kernel")
    avg_kib = sum(vals) / len(vals)
    res = dict(kernel=KERNEL, config=config, launches=len(vals), fetch_size_kib_avg=avg_kib,
               hbm_read_bytes_per_launch=2.0 * avg_kib * 1024.0,
               correction="x2: gfx950 FETCH_SIZE counts half of wide coalesced reads",
               source=os.path.relpath(path, ROOT), smx_kernels_code_sha256=kernel_sha())
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:3])
