"""bench.py — QPS of the MI355X tree-AH search path at recall@10, glove-shaped.

Workload (BASELINE.json configs[1]): glove-100-angular shape, 1,183,514 x 100
synthetic unit vectors (seeded mixture; no datasets offline), tree-AH with
1000 leaves, LUT16 AH (50 blocks x 2 dims), leaves_to_search=100, exact
reorder of 100 candidates, k=10, batch=1000 queries.  One step = one
search_batched over the 1000 device-resident queries, results written to
device memory (partition selection, LUT build, LUT16 scan + top-k, SOAR-free
dedupe, exact reorder and sort all inside the step).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config glove|sift]

`--config sift` measures BASELINE.json configs[2] (SIFT1M shape, squared L2,
2000 leaves) as a secondary line; the default is the metric's configuration.

`--gpus N` runs N ranks, one process per GPU.  Started under a launcher
(torch.distributed.run sets WORLD_SIZE), WORLD_SIZE must equal N; started
directly with N > 1, bench.py relaunches itself under
`python -m torch.distributed.run --nproc-per-node N` before anything touches
the GPU and exits with the launcher's status (`launch_plan`).  For glove /
SIFT every rank holds a replica of the index and searches its own batch of
1000 queries (queries shard with no collective: "weak" scaling); for
soar100m / deep1b the N = 8 ranks hold the 8 shards of the range split and
search one batch jointly (RangeSplitSearcher: shard search, one all-gather,
merge).  The step time is the max over ranks.  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

NQ = 1000
PARITY_QUERIES = 64
LEAVES = 1000
LEAVES_TO_SEARCH = 100
PRE_NN = 100
FINAL_NN = 10
DPB = 2


def log(msg):
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


# --config sift (BASELINE.json configs[2]) is a secondary measurement; the
# default line is configs[1], the metric's own configuration.
CONFIGS = {
    "glove": dict(n=1_183_514, leaves=1000, leaves_to_search=100, metric=0, seed=2,
                  workload="glove-100-angular shape: 1,183,514x100 dot product, tree-AH 1000 "
                           "leaves, LUT16 AH 50 blocks x 2 dims, leaves_to_search=100, reorder "
                           "100, k=10, batch=1000 queries per GPU",
                  data="synthetic (glove-100-angular-shaped seeded unit-vector mixture; no "
                       "datasets offline)",
                  metric_name="QPS at recall@10>=0.95, glove-100-angular, batch=1000; HBM GB/s achieved"),
    "sift": dict(n=1_000_000, leaves=2000, leaves_to_search=100, metric=1, seed=3,
                 workload="SIFT1M shape: 1,000,000x128 squared L2, tree + AH (non-residual) "
                          "2000 leaves, LUT16 AH 64 blocks x 2 dims, leaves_to_search=100, "
                          "reorder 100, k=10, batch=1000 queries per GPU",
                 data="synthetic (SIFT1M-shaped: 30-component low-rank mixture, |x| x 256 rounded to bytes; no "
                      "datasets offline)",
                 metric_name="QPS at recall@10, SIFT1M shape (BASELINE.json configs[2]), batch=1000"),
    # configs[3] / configs[4]: generated on the device (scann_amd/generate.py),
    # range split; at N=1 this GPU holds rank 0's shard of the `split`-way split
    "soar100m": dict(n=100_000_000, leaves=10000, leaves_to_search=100, metric=0, seed=4,
                     generated=True, split=8, soar=1.5, dim=96, components=512, spread=1.6,
                     train_sample=250_000,
                     # (k' = 2 x pre_reorder_nn per SOAR shard list: the 512-entry lists
                     # of pre 256 take the wide merge)
                     sweep=[20, 40, 60, 100, 150, 200, [100, 128], [200, 128], [400, 128],
                            [1000, 256]],
                     parity_points=[(100, 100), (200, 128), (1000, 256)],
                     workload="configs[3]: synthetic 100M x 96 dot product + SOAR (lambda 1.5, "
                              "overretrieve 2), tree-AH 10000 leaves, LUT16 AH 48 blocks x 2 "
                              "dims, leaves_to_search=100, reorder 100, k=10, batch=1000, "
                              "range split 8 ways: one rank's shard (12.5M rows, 25M members) "
                              "+ the merge of 8 shard lists",
                     data="synthetic, generated on the device (Philox per 65536-row chunk, "
                          "512 broad components (noise norm 1.6 against unit means: each "
                          "spans ~20 leaves, so recall rises with leaves_to_search), unit "
                          "norm; SURVEY §8d)",
                     metric_name="QPS per GPU of a range-split rank, configs[3] (100M x 96 "
                                 "dot + SOAR, 10000 leaves, 8-way split), batch=1000"),
    "deep1b": dict(n=1_000_000_000, leaves=50000, leaves_to_search=400, metric=0, seed=5,
                   generated=True, split=8, soar=None, dim=96, components=1 << 17,
                   train_sample=5_000_000, train_iterations=10,
                   sweep=[400, 800, 1200, 2000, [800, 256], [2000, 256], [4000, 256]],
                   parity_points=[(400, 100), (2000, 256)],
                   workload="configs[4]: Deep1B shape 1e9 x 96 dot product, tree-AH 50000 "
                            "leaves, LUT16 AH 48 blocks x 2 dims, leaves_to_search=400, reorder "
                            "100, k=10, batch=1000, dataset sharded 8 ways: one rank's shard "
                            "(125M rows) + the merge of 8 shard lists",
                   data="synthetic, generated on the device (Philox per 65536-row chunk, "
                        "131072-component unit-norm mixture; SURVEY §8d)",
                   metric_name="QPS per GPU of a range-split rank, configs[4] (Deep1B shape, "
                               "50000 leaves, 8-way shard), batch=1000"),
}
CFG = CONFIGS["glove"]
SWEEP_LEAVES = (10, 12, 15, 20, 30, 40, 50, 60, 70, 80, 100, 150)


def scan_k(num_blocks):
    """MFMA steps of the compiled scan instantiation (EffectiveKSteps in smx_searcher.hip)."""
    k = (num_blocks + 1) // 2
    return next(v for v in (4, 8, 12, 16, 20, 24, 26, 28, 32) if v >= k)


def queries_for_rank(dim, rank):
    """This rank's 1000-query batch, drawn from the dataset's own mixture."""
    from scann_amd import synthetic
    if CFG["metric"] == 0:
        return synthetic.mixture(NQ, dim, 2000, 0.9, seed=2 + 100 + 7919 * rank, means_seed=2)
    return synthetic.sift_draw(NQ, 3 + 100 + 7919 * rank, seed=3, d=dim)


def build_index(n, seed):
    from scann_amd import index_builder, synthetic
    t = time.time()
    if CFG["metric"] == 0:
        db, q = synthetic.glove_like(n=n, nq=NQ, seed=seed)
    else:
        db, q = synthetic.sift_like(n=n, nq=NQ, seed=seed)
    log(f"data {db.shape} generated in {time.time() - t:.1f}s")
    t = time.time()
    ix = index_builder.build_tree_ah(db, CFG["metric"], LEAVES, DPB, training_iterations=12,
                                     ah_training_iterations=10, seed=seed)
    sizes = ix.leaf_sizes()
    log(f"index built in {time.time() - t:.1f}s: leaves min/mean/max "
        f"{sizes.min()}/{sizes.mean():.0f}/{sizes.max()}")
    return db, q, ix


# The scan's ceiling: it issues v_smfmac_i32_32x32x64_i8, the 2:4 sparse i8
# MFMA, which covers K = 64 in the 32 cycles of the dense K = 32 form
# (tools/smfmac_chain.hip): 2 * 32 * 32 * 64 ops per 32 cycles per SIMD =
# 4096 ops/clk/SIMD x 1024 SIMDs x 2.4 GHz = 10.07 POPS "dense-equivalent" --
# twice the dense i8 peak (5 POPS, MI355X_MICROARCH.md), and exactly what
# the one-hot LUT16 GEMM needs (a one-hot row is 2:4 sparse, so the sparse
# instruction computes the whole dense product).
SMFMAC_PEAK_TOPS = 2 * 32 * 32 * 64 / 32 * 1024 * 2.4e9 / 1e12
HBM_PEAK_BPS = 8.0e12   # MI355X HBM3E (MI355X_MICROARCH.md)
DENSE_I8_PEAK_TOPS = 5000.0


def scan_roofline(code_bytes, scan_ms, timings, num_blocks):
    """roofline of the LUT16 scan kernel.  Unit of work = one (query, leaf)
    visit; SURVEY §8d's algorithmic bytes 16*B*ceil(n/32) per unit; as a
    one-hot int8 GEMM a unit is 32*ceil(n/32) datapoints x B blocks x 16
    centers x 2 ops = 64 ops per code byte.
    `frac` is against the ceiling of the instruction the kernel issues; the
    executed-instruction view (`smfmac_pipe_frac`: executed smfmac x 32
    cycles / (1024 SIMDs x 2.4 GHz x time)) also counts the padded query
    slots and K steps the kernel runs."""
    ops = 64.0 * code_bytes
    sec = scan_ms * 1e-3
    achieved = ops / sec / 1e12
    k = scan_k(num_blocks)
    # executed MFMA work: 32-slot tiles x K/2 v_smfmac_i32_32x32x64_i8 (32
    # cycles each), 16-slot tiles x 2 ceil(K/4) v_smfmac_i32_16x16x128_i8 (16)
    t32 = float(timings.get("scan_item_tiles", 0.0))
    t16 = float(timings.get("scan_item_tiles16", 0.0))
    smfmac = t32 * (k // 2)
    smfmac16 = t16 * 2 * ((k + 3) // 4)
    mfma_cycles = smfmac * 32.0 + smfmac16 * 16.0
    # useful fraction of the executed MFMA work: the algorithmic ops over the
    # dense-equivalent ops the executed instructions carry (empty query
    # slots and K padding are the rest)
    executed_ops = smfmac * 131072.0 + smfmac16 * 65536.0
    return {
        "bound": "mfma", "achieved": round(achieved, 1), "peak": round(SMFMAC_PEAK_TOPS, 1),
        "unit": "TOP/s", "frac": round(achieved / SMFMAC_PEAK_TOPS, 4),
        "peak_basis": "v_smfmac_i32_32x32x64_i8 (2:4 sparse i8 MFMA: K=64 in the 32 cycles of "
                      "the dense K=32 form) = 10.07 POPS dense-equivalent; the one-hot LUT16 "
                      "rows are exactly 2:4 sparse",
        "frac_vs_dense_i8_peak": round(achieved / DENSE_I8_PEAK_TOPS, 4),
        "kernel": f"lut16_scan_kernel<{k}> (main pass)",
        "avg_launch_ms_source": "HIP events around every scan launch, profiled replay of the "
                                "timed steps",
        "op_type": "int8 ops (TOP/s) of the one-hot LUT16 GEMM formulation",
        "algorithmic_ops_per_launch": ops,
        "algorithmic_code_bytes_per_launch": code_bytes,
        "avg_launch_ms": round(scan_ms, 5),
        "smfmac_executed_per_launch": smfmac,
        "smfmac16_executed_per_launch": smfmac16,
        "tiles_32_slot": t32, "tiles_16_slot": t16,
        "smfmac_pipe_frac": round(mfma_cycles / (1024 * 2.4e9 * sec), 4) if mfma_cycles else None,
        "useful_mfma_frac": round(ops / executed_ops, 4) if executed_ops else None,
        # SURVEY §8d's byte roofline: algorithmic code bytes / time; above the
        # 8 TB/s HBM peak by design (the query tiles of a leaf re-read its
        # codes from L2), hence the MFMA bound
        "code_GBps_algorithmic": round(code_bytes / sec / 1e9, 1),
        # secondary: LUT16 lookups per second; 16*B bytes hold
        # 32 datapoints x B codes -> 2 lookups per byte
        "lookups_per_s": round(2.0 * code_bytes / sec, 1),
    }


def kernel_source_sha():
    """sha256 of scann_amd/csrc/smx_kernels.hip with // and /* */ comments and
    all blank space removed: the code a traffic record was measured on."""
    import hashlib
    import re
    with open(os.path.join(ROOT, "scann_amd", "csrc", "smx_kernels.hip")) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    src = re.sub(r"\s+", "", src)
    return hashlib.sha256(src.encode()).hexdigest()


def scan_traffic(config):
    """HBM read bytes per scan launch from this config's own PMC FETCH_SIZE
    pass (tools/profile_bench.sh -> tools/pmc_traffic.py ->
    profiles/scan_traffic_<config>.json), only when it was measured on the
    same kernel source; None otherwise."""
    tpath = os.path.join(ROOT, "profiles", f"scan_traffic_{config}.json")
    if not os.path.exists(tpath):
        return None
    with open(tpath) as f:
        tr = json.load(f)
    if kernel_source_sha() != tr.get("smx_kernels_code_sha256"):
        return None
    return tr["hbm_read_bytes_per_launch"]


def cpu_info():
    """CPU model and SIMD ISA of the host (lscpu's fields, from /proc/cpuinfo)."""
    model, flags = "unknown", set()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name") and model == "unknown":
                    model = line.split(":", 1)[1].strip()
                elif line.startswith("flags") and not flags:
                    flags = set(line.split(":", 1)[1].split())
    except OSError:
        pass
    isa = [x for x in ("sse4_2", "avx", "avx2", "fma", "avx512f", "avx512bw", "avx512_vnni",
                       "avx512_vbmi") if x in flags]
    return model, isa


def host_threads():
    """(cores this process can use, cores in its affinity mask): the affinity
    mask capped by a cgroup CPU quota (a shared host grants a share of its
    cores; threads beyond it only time-slice)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    cores = aff
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()[:2]),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", None)):
        try:
            with open(path) as f:
                text = f.read()
            if parse is not None:
                quota, period = parse(text)
            else:
                quota = text.strip()
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                    period = f.read().strip()
            if quota not in ("max", "-1"):
                cores = max(1, min(aff, int(float(quota) / float(period))))
            break
        except (OSError, ValueError):
            continue
    return cores, aff


def cpu_baseline(ix, q, gpu_idx, threads):
    """The oracle's AVX2 port of the reference path on all host cores (rank 0):
    median of 5 timed runs, each >= 2 s of repeated 1000-query batches, with the
    leaf-scan phase (LUT16 + FastTopNeighbors) timed on its own."""
    from oracle import binding as oracle
    oracle.build()
    try:
        port = oracle.Avx2Port(ix)
    except ValueError:   # residual without the global top-N path: the C restatement
        return cpu_baseline_restatement(ix, q, gpu_idx, threads)
    pipeline = ("pipeline A: tree_ah_hybrid_residual.cc batched path, leaves in "
                "leaf_tokens_by_norm_ order, int16 truncated prefilter over the global "
                "FastTopNeighbors" if ix.residual else
                "pipeline B: tree_x_hybrid_smmd.cc optimized batched path, leaves in ascending "
                "id, per-leaf FastTopNeighbors<int16_t> with the global epsilon at visit time, "
                "merged into the global FastTopNeighbors<float>")
    model, isa = cpu_info()
    port.search(q, LEAVES_TO_SEARCH, PRE_NN, FINAL_NN, True, threads)  # warm-up + calibration
    t = time.perf_counter()
    out = port.search(q, LEAVES_TO_SEARCH, PRE_NN, FINAL_NN, True, threads)
    per_batch = time.perf_counter() - t
    reps = max(1, int(np.ceil(2.0 / max(per_batch, 1e-3))))
    _, aff = host_threads()

    def timed_runs(n_runs, shared):
        runs, scan_runs, front_runs, res = [], [], [], None
        for _ in range(n_runs):
            t_total, scan_s, front_s = 0.0, 0.0, 0.0
            for _ in range(reps):
                t = time.perf_counter()
                res = port.search(q, LEAVES_TO_SEARCH, PRE_NN, FINAL_NN, True, threads,
                                  batch_shared=shared)
                t_total += time.perf_counter() - t
                scan_s += port.last_phase_s["scan"]
                front_s += port.last_phase_s["front"]
            nqs = reps * q.shape[0]
            runs.append(nqs / t_total)
            # a phase's CPU seconds spread over the cores
            scan_runs.append(nqs * threads / max(scan_s, 1e-9))
            front_runs.append(nqs * threads / max(front_s, 1e-9))
        return runs, scan_runs, front_runs, res

    # the reference's bottom loop (codes shared by a batch's <= 3 queries,
    # kSmart prefetch) is the baseline; the round-2 per-query loop beside it
    runs, scan_runs, front_runs, out = timed_runs(5, True)
    _, scan_runs_pq, _, _ = timed_runs(3, False)
    # the port replays the reference's emulate semantics; the GPU computes the
    # ideal exact top-k', so this is the emulate-vs-GPU id mismatch
    mismatch = float((out[0] != gpu_idx).mean())
    port.close()
    return dict(value=round(float(np.median(runs)), 1), unit="queries/s", cores=threads,
                affinity_cores=aff, kind="port", cpu_model=model, isa=isa,
                runs_qps=[round(x, 1) for x in runs],
                scan_only_qps=round(float(np.median(scan_runs)), 1),
                scan_only_qps_per_query_loop=round(float(np.median(scan_runs_pq)), 1),
                front_only_qps=round(float(np.median(front_runs)), 1),
                sample=f"median of 5 runs x {reps} repeats of the same {q.shape[0]}-query batch "
                       f"through the AVX2 port of the reference's batched tree-AH path "
                       f"({pipeline}; oracle/lut16_avx2_port.cc: SearchBatchedParallel chunking, "
                       f"the reference's Avx2LUT16BottomLoop (pshufb LUT16 with the codes of a "
                       f"32-datapoint group shared by the <= 3 queries of a batch, tag-along "
                       f"int16 accumulation, kSmart next-partition prefetch), emulate-mode "
                       f"FastTopNeighbors, "
                       f"partition scores "
                       f"8 centers per AVX2 vector in the many-to-many order), {threads} threads "
                       f"= every core this process may use ({aff} in its affinity mask, capped "
                       f"by the cgroup CPU quota); scan_only_qps = the leaf scan phase alone "
                       f"(its CPU seconds / cores); scan_only_qps_per_query_loop = the same "
                       f"with one group pass per query (the round-2 port)",
                id_mismatch_vs_gpu=mismatch)


def cpu_baseline_restatement(ix, q, gpu_idx, threads):
    """Indexes the AVX2 port does not cover: the oracle's scalar C restatement
    (ideal mode), multithreaded over queries."""
    from oracle import binding as oracle
    reps, t_total, out = 0, 0.0, None
    while reps < 50 and (t_total < 10.0 or reps == 0):
        t = time.perf_counter()
        out = oracle.search(ix, q, LEAVES_TO_SEARCH, PRE_NN, FINAL_NN, True, oracle.MODE_IDEAL,
                            threads)
        t_total += time.perf_counter() - t
        reps += 1
    return dict(value=round(reps * q.shape[0] / t_total, 1), unit="queries/s", cores=threads,
                kind="port",
                sample=f"{reps} x the same {q.shape[0]}-query batch through the oracle's scalar "
                       f"C restatement (oracle/scann_oracle.cc, ideal mode; the AVX2 port covers "
                       f"the residual global top-N path only), {threads} threads, {t_total:.1f}s",
                id_mismatch_vs_gpu=float((out[0] != gpu_idx).mean()))


def launch_plan(gpus, env, argv, port=None):
    """What `bench.py --gpus N` does before touching the GPU:
    ("run", world) -- run as one rank of `world` (WORLD_SIZE, or 1);
    ("relaunch", cmd) -- N > 1 with no launcher: start N ranks with
    torch.distributed.run (rendezvous on 127.0.0.1) and exit with its status;
    ("error", message) -- --gpus disagrees with the launcher's WORLD_SIZE."""
    if gpus < 1:
        return ("error", f"--gpus must be >= 1 (got {gpus})")
    world_env = env.get("WORLD_SIZE")
    if world_env is None:
        if gpus == 1:
            return ("run", 1)
        if port is None:
            import socket
            with socket.socket() as sk:
                sk.bind(("127.0.0.1", 0))
                port = sk.getsockname()[1]
        return ("relaunch", [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                             f"--nproc-per-node={gpus}", "--master-addr=127.0.0.1",
                             f"--master-port={port}", os.path.abspath(__file__)] + list(argv))
    if int(world_env) != gpus:
        return ("error", f"--gpus {gpus} but the launcher started WORLD_SIZE={world_env} ranks")
    return ("run", gpus)


def main():
    plan = launch_plan(_peek_gpus(sys.argv[1:]), os.environ, sys.argv[1:])
    if plan[0] == "error":
        print(f"bench.py: {plan[1]}", file=sys.stderr)
        sys.exit(2)
    if plan[0] == "relaunch":
        # a child process, not exec: this process has not touched the GPU
        import subprocess
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        sys.exit(subprocess.call(plan[1], env=env))
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--n", type=int, default=1_183_514)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="glove")
    ap.add_argument("--no-sweep", action="store_true",
                    help="skip the leaves_to_search QPS-recall operating points")
    ap.add_argument("--sweep-steps", type=int, default=20)
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the oracle check of the generated-shard lines")
    ap.add_argument("--leaves-to-search", type=int, default=0,
                    help="override the configuration's leaves_to_search (0: as configured)")
    ap.add_argument("--no-latency", action="store_true",
                    help="skip the one-batch-at-a-time timing (the per-batch latency)")
    ap.add_argument("--no-stages", action="store_true",
                    help="skip the per-stage replay (stage_ms, the scan alone)")
    ap.add_argument("--in-flight", type=int, default=3,
                    help="query batches in flight (streams, one library workspace each)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak",
                    help="weak: every GPU searches its own 1000-query batches (value); strong: "
                         "one 1000-query batch split over the GPUs, results all-gathered "
                         "(value); the other mode is reported beside it when N > 1")
    args = ap.parse_args()
    global CFG, LEAVES, LEAVES_TO_SEARCH
    CFG = CONFIGS[args.config]
    LEAVES, LEAVES_TO_SEARCH = CFG["leaves"], args.leaves_to_search or CFG["leaves_to_search"]
    if args.config != "glove" and args.n == 1_183_514:
        args.n = CFG["n"]

    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # rehearsal of the N-rank paths on a one-GPU box (never the measured
    # configuration): SMX_BENCH_ONE_DEVICE=1 puts every rank on device 0,
    # SMX_BENCH_BACKEND=gloo avoids RCCL's one-rank-per-GPU rule
    if os.environ.get("SMX_BENCH_ONE_DEVICE") == "1":
        local = 0
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(os.environ.get("SMX_BENCH_BACKEND") or
                                ("nccl" if torch.cuda.is_available() else "gloo"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    if CFG.get("generated"):
        return main_generated(args, rank, world, local, dist, dev)

    from scann_amd import _native, synthetic
    db, _, ix = build_index(args.n, seed=CFG["seed"])
    # per-rank query batch from the same mixture (weak scaling)
    q = queries_for_rank(db.shape[1], rank)
    nat = _native.NativeIndex(ix, device=local)
    log(f"native index: {nat.info()}")

    qd = torch.from_numpy(q).to(dev)
    # batches in flight: step i runs on stream i % in_flight with its own
    # output buffers; the library keeps one workspace per stream, so two
    # consecutive batches overlap on the device (one's latency-bound front end
    # and select beside the other's scan) -- whole-job throughput, every
    # batch searched completely; the single-stream rate is reported beside it
    n_fl = max(1, args.in_flight)
    # (SMX_BENCH_STREAM_PRIORITY="-1,0,0": per-stream priorities, an A/B knob)
    prio = [int(x) for x in os.environ.get("SMX_BENCH_STREAM_PRIORITY", "").split(",") if x]
    streams = [torch.cuda.Stream(dev, priority=prio[i % len(prio)] if prio else 0)
               for i in range(n_fl)]
    outs = [(torch.zeros((NQ, FINAL_NN), dtype=torch.int32, device=dev),
             torch.zeros((NQ, FINAL_NN), dtype=torch.float32, device=dev),
             torch.zeros(NQ, dtype=torch.int32, device=dev)) for _ in range(n_fl)]
    out_idx, out_dist, out_cnt = outs[0]
    torch.cuda.synchronize()

    def step(i=0, leaves=LEAVES_TO_SEARCH, fl=None):
        k = i % (fl or n_fl)
        o = outs[k]
        nat.search_batched_device(qd.data_ptr(), NQ, leaves, PRE_NN, FINAL_NN, True,
                                  o[0].data_ptr(), o[1].data_ptr(), o[2].data_ptr(),
                                  stream=ctypes.c_void_p(streams[k].cuda_stream))

    enqueue_s, wall_s = {}, {}

    def timed_steps(fl, fn=None):
        """K steps bracketed by barrier + synchronize; the elapsed time is
        taken from HIP events (recorded on streams[0] after the bracket's
        synchronize, every stream waiting on it, and after joining every
        stream), so host jitter outside the device's work does not enter it;
        the wall clock of the same bracket is kept beside it.  Max over
        ranks."""
        fn = fn or (lambda i: step(i, fl=fl))
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(streams[0])
        for st in streams[1:]:
            st.wait_event(e0)
        for i in range(args.steps):
            fn(i)
        for st in streams[1:]:
            streams[0].wait_stream(st)
        e1.record(streams[0])
        enqueue_s[fl] = time.perf_counter() - t0   # host time issuing the steps
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        el = e0.elapsed_time(e1) * 1e-3
        if dist is not None:
            tt = torch.tensor([el, wall], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el, wall = float(tt[0].item()), float(tt[1].item())
        wall_s[fl] = wall
        return el

    # timed steps: eager launches of the pipeline kernels per step
    nat.set_profiling(False)
    for i in range(max(args.warmup, n_fl)):
        step(i)
    elapsed = timed_steps(n_fl)
    wall_ms_per_step = wall_s[n_fl] * 1000.0 / args.steps
    ms_per_step = elapsed * 1000.0 / args.steps
    # host time spent issuing the timed steps (library calls, launches): when
    # it nears ms_per_step the host, not the device, sets the rate
    issue_ms = enqueue_s[n_fl] * 1000.0 / args.steps
    value = world * NQ * args.steps / elapsed
    # the same in-flight steps again with two HIP events around every scan
    # launch on its own stream (profiling mode 2: no synchronisation, the
    # batches stay in flight): the roofline's per-launch scan duration, and
    # the rate with the events (their host cost is kept out of `value`)
    nat.set_profiling(2)
    elapsed_ev = timed_steps(n_fl)
    t_fl = nat.timings()
    nat.set_profiling(False)
    scan_ms_fl, scan_launches = float(t_fl["scan_ms_mode2"]), int(t_fl["scan_launches"])
    # the same steps one at a time (one stream): the per-batch latency
    elapsed_1 = timed_steps(1) if n_fl > 1 and not args.no_latency else None

    # strong scaling: rank 0's 1000-query batch split over
    # the ranks by query_slice (SearchBatchedParallel's chunking,
    # scann.cc:478-501, across GPUs), each slice searched on the step's
    # stream and the slices' results all-gathered (RCCL), so every rank holds
    # the whole batch's results; QPS = 1000 x K / max-rank time
    strong = None
    if world > 1 or args.scaling == "strong":
        from scann_amd.distributed import SplitBatchSearcher, query_slice
        q0d = qd if rank == 0 else torch.from_numpy(queries_for_rank(db.shape[1], 0)).to(dev)
        b0, e0_ = query_slice(NQ, rank, world)
        souts = [(torch.zeros((e0_ - b0, FINAL_NN), dtype=torch.int32, device=dev),
                  torch.zeros((e0_ - b0, FINAL_NN), dtype=torch.float32, device=dev),
                  torch.zeros(e0_ - b0, dtype=torch.int32, device=dev)) for _ in range(n_fl)]
        gathered = [None] * n_fl

        def strong_step(i):
            k = i % n_fl
            o = souts[k]

            def search(qs):
                nat.search_batched_device(qs.data_ptr(), int(qs.shape[0]), LEAVES_TO_SEARCH,
                                          PRE_NN, FINAL_NN, True, o[0].data_ptr(),
                                          o[1].data_ptr(), o[2].data_ptr(),
                                          stream=ctypes.c_void_p(streams[k].cuda_stream))
                return o

            with torch.cuda.stream(streams[k]):
                gathered[k] = SplitBatchSearcher(search, rank, world, None).search_batched(q0d)

        for i in range(max(args.warmup, n_fl)):
            strong_step(i)
        el_s = timed_steps(n_fl, strong_step)
        torch.cuda.synchronize()
        strong = {"qps": round(NQ * args.steps / el_s, 1),
                  "ms_per_step": round(el_s * 1000.0 / args.steps, 4),
                  "queries_per_gpu": e0_ - b0,
                  "parallelism": f"one {NQ}-query batch split over {world} GPU(s) by query_slice, "
                                 f"results all-gathered"
                                 + ((" (RCCL all_gather_into_tensor)"
                                     if dist.get_backend() == "nccl"
                                     else f" ({dist.get_backend()} all_gather)")
                                    if world > 1 else "")
                                 + f", {n_fl} batches in flight"}
        if rank == 0:
            # the split result == the whole batch searched on one GPU (rank 0's
            # weak-scaling batch is the same queries)
            g = gathered[(args.steps - 1) % n_fl]
            whole = outs[(args.steps - 1) % n_fl] if args.steps else outs[0]
            strong["ids_equal_whole_batch"] = bool(torch.equal(g[0], whole[0]))

    # per-stage durations, each kernel alone: the same steps replayed one at
    # a time with HIP events recorded on the call's stream around every stage
    # launch (profiling mode 1: synchronous calls); with --no-stages one such
    # call only, for the launch's code bytes and tile counts
    nat.set_profiling(True)
    step()
    scan_ms, stage, scan_bytes = [], {}, []
    n_rep = 1 if args.no_stages else args.steps
    for _ in range(n_rep):
        step()
        t = nat.timings()
        scan_ms.append(t["scan_ms"])
        scan_bytes.append(t["scan_code_bytes"])
        for k in ("partition_ms", "lut_ms", "invert_ms", "seed_scan_ms", "seed_select_ms",
                  "scan_ms", "select_ms", "total_ms"):
            stage[k] = stage.get(k, 0.0) + t[k] / n_rep
    t_last = nat.timings()
    nat.set_profiling(False)
    torch.cuda.synchronize()

    # recall@10 of this rank's batch against exact brute force
    gidx = out_idx.cpu().numpy().astype(np.int64)
    truth = synthetic.brute_force_topk(db, q, FINAL_NN, CFG["metric"])
    recall = synthetic.recall_at_k(gidx, truth, FINAL_NN)

    # QPS-recall operating points (QPS at the smallest
    # leaves_to_search reaching recall@10 >= 0.95); the headline value stays
    # at the configured leaves_to_search.  Same batch, same timing method.
    points = []
    if not args.no_sweep:
        for lv in SWEEP_LEAVES:
            if lv > LEAVES:
                continue
            for i in range(3):
                step(i, lv)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for i in range(args.sweep_steps):
                step(i, lv)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            r = synthetic.recall_at_k(out_idx.cpu().numpy().astype(np.int64), truth, FINAL_NN)
            points.append({"leaves_to_search": lv, "qps": round(NQ * args.sweep_steps / dt, 1),
                           "recall_at_10": round(r, 4)})
        step()
        torch.cuda.synchronize()

    avg_scan_ms = float(np.mean(scan_ms))
    bytes_per_launch = float(np.mean(scan_bytes))
    # the roofline of the scan kernel alone on the device (serial replay, HIP
    # events around each scan launch: the duration rocprofv3 reports for one
    # batch at a time, profiles/r06/prof_*_alone/), and beside it the launches
    # of the timed region, which share the device with the other batches in
    # flight (their duration is residency, not the kernel's own time)
    roof = scan_roofline(bytes_per_launch, avg_scan_ms, t_last, ix.num_blocks)
    roof["avg_launch_ms_source"] = (
        f"HIP events on the call's stream around the scan of {len(scan_ms)} calls replayed one "
        f"at a time (the kernel alone on the device)")
    fl = scan_roofline(bytes_per_launch, scan_ms_fl, t_last, ix.num_blocks)
    roof["in_flight"] = {
        "avg_launch_ms": fl["avg_launch_ms"], "achieved": fl["achieved"], "frac": fl["frac"],
        "smfmac_pipe_frac": fl["smfmac_pipe_frac"],
        # scans resident at once on average: launch time x launches / elapsed
        "scan_concurrency": round(scan_ms_fl * 1e-3 * args.steps / elapsed_ev, 3),
        "source": f"HIP events on each call's stream around every scan launch of a second timed "
                  f"pass of the same in-flight steps ({scan_launches} launches, {n_fl} batches "
                  f"in flight, {world * NQ * args.steps / elapsed_ev:.0f} QPS with the events): "
                  f"each launch shares the device with the other batches' kernels"}
    traffic = scan_traffic(args.config)

    if rank == 0:
        result = {
            "metric": CFG["metric_name"],
            "value": round(value, 1),
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "in_flight": n_fl,
            "host_issue_ms_per_step": round(issue_ms, 4),
            "single_stream": ({"qps": round(world * NQ * args.steps / elapsed_1, 1),
                               "ms_per_step": round(elapsed_1 * 1000.0 / args.steps, 4)}
                              if elapsed_1 else None),
            "timing": "HIP events between the timed region's barrier + synchronize brackets "
                      "(max over ranks); wall clock of the same brackets: "
                      f"{wall_ms_per_step:.4f} ms/step",
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int8",
            "data": CFG["data"],
            "config": {
                "workload": CFG["workload"],
                "num_datapoints": int(args.n), "dim": int(db.shape[1]), "num_leaves": LEAVES,
                "leaves_to_search": LEAVES_TO_SEARCH, "pre_reorder_nn": PRE_NN,
                "final_nn": FINAL_NN, "batch": NQ,
                "parallelism": f"query-sharded replicas x{world}, {n_fl} batches in flight per GPU",
            },
            "recall_at_10": round(recall, 4),
            "roofline": dict(roof, traffic=traffic,
                             hbm_GBps_measured=(round(traffic / (avg_scan_ms * 1e-3) / 1e9, 1)
                                                if traffic else None),
                             # the scan's HBM basis: PMC bytes per launch / the kernel alone /
                             # 8 TB/s (MI355X_MICROARCH.md)
                             hbm_frac=(round(traffic / (avg_scan_ms * 1e-3) / HBM_PEAK_BPS, 4)
                                       if traffic else None)),
            "stage_ms": ({k: round(v, 4) for k, v in stage.items()} if not args.no_stages
                         else None),
            "operating_points": points,
            "qps_at_recall_0.95": next(({"leaves_to_search": p["leaves_to_search"],
                                         "qps": p["qps"], "recall_at_10": p["recall_at_10"]}
                                        for p in points if p["recall_at_10"] >= 0.95), None),
            "candidates_max": t_last["max_candidates"],
            "candidates_mean": round(float(t_last["mean_candidates"]), 1),
        }
        if strong is not None:
            if args.scaling == "strong":
                # the split batch is the line's value; the weak figures beside it
                result["weak_scaling"] = {"qps": result["value"],
                                          "ms_per_step": result["ms_per_step"],
                                          "parallelism": result["config"]["parallelism"]}
                result["value"] = strong["qps"]
                result["ms_per_step"] = strong["ms_per_step"]
                result["scaling"] = "strong"
                result["config"]["batch"] = NQ
                result["config"]["parallelism"] = strong["parallelism"]
                result["strong_scaling"] = {k: v for k, v in strong.items()
                                            if k not in ("qps", "ms_per_step", "parallelism")}
            else:
                result["strong_scaling"] = strong
        # full-size parity: oracle (ideal mode) on a query subset, ids must match
        from oracle import binding as oracle
        oracle.build()
        sub = 64
        oi, od, _ = oracle.search(ix, q[:sub], LEAVES_TO_SEARCH, PRE_NN, FINAL_NN, True,
                                  oracle.MODE_IDEAL, min(16, os.cpu_count() or 1))
        gsub = out_idx[:sub].cpu().numpy().astype(np.uint32)
        gds = out_dist[:sub].cpu().numpy()
        result["parity_vs_oracle"] = {
            "queries": sub, "id_mismatch": float((oi != gsub).mean()),
            "max_rel_dist_err": float(np.max(np.abs(gds - od) / np.maximum(np.abs(od), 1e-30))),
        }
        if not args.no_cpu_baseline:
            threads = args.cpu_threads or host_threads()[0]
            log(f"cpu baseline with {threads} threads ...")
            result["cpu_baseline"] = cpu_baseline(ix, q, out_idx.cpu().numpy().astype(np.uint32),
                                                  threads)
        print(json.dumps(result), flush=True)
    nat.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def main_generated(args, rank, world, local, dist, dev):
    """configs[3]/[4]: rank `rank` of a `split`-way range split, its shard
    generated and built on this GPU.  With world == split the ranks run the
    real split (shard search, one all-gather, merge on every rank); with
    world == 1 this GPU is rank 0 of the split and the merge runs over `split`
    copies of its shard list (the all-gather's shape; the xGMI all-gather
    itself is not in the single-GPU step)."""
    import torch
    from scann_amd import generate, synthetic
    from scann_amd.distributed import NativeShardEngine, RangeSplitSearcher, all_gather_entries
    split = CFG["split"]
    if world not in (1, split):
        raise SystemExit(f"--config {args.config}: run with 1 or {split} ranks")
    shard_rank = rank if world == split else 0
    n = args.n if args.n != 1_183_514 else CFG["n"]
    t = time.time()
    ds = generate.GeneratedDataset(n, CFG["dim"], CFG["seed"], components=CFG["components"],
                                   spread=CFG.get("spread", 0.9), device=dev)
    torch.cuda.synchronize()
    t_build = time.perf_counter()
    ix = generate.build_generated_shard(
        ds, LEAVES, shard_rank, split, soar_lambda=CFG["soar"], seed=CFG["seed"],
        training_sample_size=CFG.get("train_sample", max(250_000, 20 * LEAVES)),
        training_iterations=CFG.get("train_iterations", 8),
        counts_from_all_ranks=False, log=log)
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t_build
    log(f"shard {shard_rank}/{split} built in {build_s:.1f}s (generation included): "
        f"{ix.num_members} members")
    q = ds.queries(NQ, CFG["seed"] + 1000)
    eng = NativeShardEngine(ix, device=local)
    qd = torch.from_numpy(q).to(dev)
    k = eng.shard_width(LEAVES_TO_SEARCH, PRE_NN, FINAL_NN, True)
    # batches in flight (one rank of the split on one GPU only; the 8-rank
    # step keeps one, its all-gather ordering the ranks)
    n_fl = max(1, args.in_flight) if world == 1 else 1
    fl_streams = [torch.cuda.Stream(dev) for _ in range(n_fl)]
    local_es = [torch.empty((NQ, k, 2), dtype=torch.int64, device=dev) for _ in range(n_fl)]
    gathereds = [torch.empty((split, NQ, k, 2), dtype=torch.int64, device=dev) for _ in range(n_fl)]
    local_e, gathered = local_es[0], gathereds[0]
    res = {}
    ctr = [0]

    def search(slot=0):
        eng.search_shard(qd, LEAVES_TO_SEARCH, PRE_NN, FINAL_NN, True, local_es[slot])

    def merge(slot=0):
        if world == split:
            g = all_gather_entries(local_es[slot], world)
        else:
            gathereds[slot].copy_(local_es[slot].unsqueeze(0).expand_as(gathereds[slot]))
            g = gathereds[slot]
        res["out"] = eng.merge(split, g, NQ, LEAVES_TO_SEARCH, PRE_NN, FINAL_NN, True)

    def timed(fn, steps):
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if dist is not None:
            tt = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt.item())
        return el

    # the N-rank step is the searcher the distributed module exports
    # (RangeSplitSearcher: shard search, one all-gather, merge on every rank)
    searcher = RangeSplitSearcher(eng, world) if world == split else None

    def step():
        if searcher is not None:
            res["out"] = searcher.search_batched(qd, LEAVES_TO_SEARCH, PRE_NN, FINAL_NN, True)
        elif n_fl == 1:
            search()
            merge()
        else:   # step i on stream i % n_fl (its own shard list and merge buffers)
            slot = ctr[0] % n_fl
            ctr[0] += 1
            with torch.cuda.stream(fl_streams[slot]):
                search(slot)
                merge(slot)

    for _ in range(args.warmup):
        step()
    elapsed = timed(step, args.steps)
    search_s = timed(search, args.steps)
    merge_s = timed(merge, args.steps)
    ms_per_step = elapsed * 1000.0 / args.steps
    # recall@10 of rank 0's merged result against exact brute force over the
    # rows the split's ranks hold (world == 1: this shard's rows)
    nat = eng.nat
    nat.set_profiling(True)
    search()
    scan_ms, scan_bytes = [], []
    for _ in range(min(args.steps, 20)):
        search()
        tm = nat.timings()
        scan_ms.append(tm["scan_ms"])
        scan_bytes.append(tm["scan_code_bytes"])
    stages = nat.timings()
    nat.set_profiling(False)
    step()
    torch.cuda.synchronize()
    if world == 1:   # this rank's own result (the timed merge saw duplicated lists)
        res["out"] = eng.merge(1, local_e.unsqueeze(0), NQ, LEAVES_TO_SEARCH, PRE_NN, FINAL_NN,
                               True)
    gidx = res["out"][0].cpu().numpy().astype(np.int64)
    c0, c1 = ds.chunk_range(shard_rank, split) if world == 1 else (0, ds.num_chunks)
    r0, r1 = c0 * generate.CHUNK, min(c1 * generate.CHUNK, n)
    truth = _generated_truth(ds, q, r0, r1, dev)
    recall = synthetic.recall_at_k(gidx, truth, FINAL_NN)
    # QPS-recall operating points over leaves_to_search (the headline value
    # stays at the configured one): search + merge timed as above, recall of
    # this rank's merged result
    points = []
    if not args.no_sweep:
        for sw in CFG.get("sweep", []):
            lv, pre = (sw, PRE_NN) if isinstance(sw, int) else (sw[0], sw[1])
            if lv > LEAVES:
                continue
            kl = eng.shard_width(lv, pre, FINAL_NN, True)
            le = torch.empty((NQ, kl, 2), dtype=torch.int64, device=dev)
            gl = torch.empty((split, NQ, kl, 2), dtype=torch.int64, device=dev)

            def sweep_step():
                eng.search_shard(qd, lv, pre, FINAL_NN, True, le)
                if world == split:
                    g = all_gather_entries(le, world)
                else:
                    gl.copy_(le.unsqueeze(0).expand_as(gl))
                    g = gl
                return eng.merge(split, g, NQ, lv, pre, FINAL_NN, True)

            for _ in range(2):
                sweep_step()
            el = timed(sweep_step, max(2, args.sweep_steps // 2))
            eng.search_shard(qd, lv, pre, FINAL_NN, True, le)
            own = eng.merge(1, le.unsqueeze(0), NQ, lv, pre, FINAL_NN, True)
            r = synthetic.recall_at_k(own[0].cpu().numpy().astype(np.int64), truth, FINAL_NN)
            points.append({"leaves_to_search": lv, "pre_reorder_nn": pre,
                           "qps": round(NQ * max(2, args.sweep_steps // 2) / el, 1),
                           "recall_at_10": round(r, 4)})
            del le, gl
    avg_scan_ms = float(np.mean(scan_ms))
    bytes_per_launch = float(np.mean(scan_bytes))
    roof = scan_roofline(bytes_per_launch, avg_scan_ms, stages, ix.num_blocks)
    traffic = scan_traffic(args.config)
    if rank == 0:
        result = {
            "metric": CFG["metric_name"],
            # the ranks search the same batch jointly: whole-job QPS
            "value": round(NQ * args.steps / elapsed, 1),
            "unit": "queries/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4), "in_flight": n_fl, "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None, "dtype": "int8", "data": CFG["data"],
            "config": {"workload": CFG["workload"], "num_datapoints": n, "dim": CFG["dim"],
                       "num_leaves": LEAVES, "leaves_to_search": LEAVES_TO_SEARCH,
                       "pre_reorder_nn": PRE_NN, "final_nn": FINAL_NN, "batch": NQ,
                       "split": split, "shard_members": int(ix.num_members),
                       "parallelism": (f"range split x{split}" if world == split else
                                       f"rank 0 of a {split}-way range split on 1 GPU, "
                                       f"{n_fl} batches in flight")},
            "recall_at_10": round(recall, 4),
            "recall_reference": ("exact brute force over the shard's rows" if world == 1
                                 else "exact brute force over the whole dataset"),
            "operating_points": points,
            "qps_at_recall_0.95": max(({"leaves_to_search": p["leaves_to_search"],
                                        "pre_reorder_nn": p["pre_reorder_nn"], "qps": p["qps"],
                                        "recall_at_10": p["recall_at_10"]}
                                       for p in points if p["recall_at_10"] >= 0.95),
                                      key=lambda p: p["qps"], default=None),
            "build_s": round(build_s, 2),
            "build": ("generation + the whole shard build on this GPU in the HIP build kernels "
                      "(k-means on a %d-row sample, tokenization%s, grouping, codebook, codes)"
                      % (CFG.get("train_sample", max(250_000, 20 * LEAVES)),
                         " + SOAR" if CFG["soar"] else "")),
            "shard_search_ms": round(search_s * 1000.0 / args.steps, 4),
            "merge_ms": round(merge_s * 1000.0 / args.steps, 4),
            "merge_input": (f"all-gather of {split} ranks" if world == split else
                            f"{split} copies of this rank's [nq][{k}] list"),
            "roofline": dict(roof, traffic=traffic,
                             hbm_GBps_measured=(round(traffic / (avg_scan_ms * 1e-3) / 1e9, 1)
                                                if traffic else None),
                             # the scan's HBM basis: PMC bytes per launch / the kernel alone /
                             # 8 TB/s (MI355X_MICROARCH.md)
                             hbm_frac=(round(traffic / (avg_scan_ms * 1e-3) / HBM_PEAK_BPS, 4)
                                       if traffic else None)),
            "stage_ms": {k2: round(stages[k2], 4) for k2 in
                         ("partition_ms", "invert_ms", "seed_scan_ms", "scan_ms", "select_ms",
                          "total_ms")},
        }
        view_ids = None
        if not args.no_parity:
            result["parity_vs_oracle"], view_ids = shard_parity(
                ix, eng, q, CFG["parity_points"], args.cpu_threads or host_threads()[0], local)
        if not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline_shard(ix, q, args.cpu_threads or host_threads()[0],
                                                        view_ids)
        print(json.dumps(result), flush=True)
    nat.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def _generated_truth(ds, q, r0, r1, dev):
    """Exact top-k ids (float64 scores) over generated rows [r0, r1)."""
    import torch
    from scann_amd import generate
    qt = torch.from_numpy(q).to(dev, torch.float64)
    best_s = torch.full((q.shape[0], FINAL_NN), float("inf"), dtype=torch.float64, device=dev)
    best_i = torch.zeros((q.shape[0], FINAL_NN), dtype=torch.int64, device=dev)
    for c in range(r0 // generate.CHUNK, (r1 + generate.CHUNK - 1) // generate.CHUNK):
        x = ds.chunk(c).to(torch.float64)
        sc = -(qt @ x.T)
        s = torch.cat([best_s, sc], 1)
        i = torch.cat([best_i, torch.arange(c * generate.CHUNK, c * generate.CHUNK + x.shape[0],
                                            device=dev).expand(q.shape[0], -1)], 1)
        v, j = torch.topk(s, FINAL_NN, dim=1, largest=False)
        best_s, best_i = v, torch.gather(i, 1, j)
    return best_i.cpu().numpy()


def shard_parity(ix, eng, q, points, threads, device):
    """parity_vs_oracle of a shard line at workload size, per (leaves_to_search,
    pre_reorder_nn) point on PARITY_QUERIES queries:
    * the benchmarked path itself -- this rank's shard engine (search_shard +
      the merge of its one list) -- against the oracle (ideal mode) on the
      shard: the whole index's ties (leaf << shift | leaf_row_base + row),
      spill factor and SOAR dedupe, the reorder from the members' own rows;
      global ids and distance bits must be equal;
    * the shard viewed as a standalone index (TreeAHIndex.standalone: members
      renumbered, a SOAR shard's copies distinct) through search_batched
      against the oracle on that view."""
    import torch
    from oracle import binding as oracle
    from scann_amd import _native
    oracle.build()
    view = ix.standalone()
    sub = q[:PARITY_QUERIES]
    nv = _native.NativeIndex(view, device=device)
    out = []
    view_ids = {}
    try:
        for lv, pre in points:
            t = time.perf_counter()
            oi, od, oc = oracle.search(ix, sub, lv, pre, FINAL_NN, True, oracle.MODE_IDEAL, threads)
            qd = torch.from_numpy(sub).to(eng.device)
            k = eng.shard_width(lv, pre, FINAL_NN, True)
            le = torch.empty((sub.shape[0], k, 2), dtype=torch.int64, device=eng.device)
            eng.search_shard(qd, lv, pre, FINAL_NN, True, le)
            si, sd, sc = eng.merge(1, le.unsqueeze(0), sub.shape[0], lv, pre, FINAL_NN, True)
            torch.cuda.synchronize()
            si = si.cpu().numpy().astype(np.uint32)
            sd = sd.cpu().numpy()
            sc = sc.cpu().numpy()
            ent = {"leaves_to_search": lv, "pre_reorder_nn": pre, "queries": int(sub.shape[0]),
                   "id_mismatch": float((si != oi).mean()),
                   "dist_bits_mismatch": float((sd.view(np.uint32) != od.view(np.uint32)).mean()),
                   "count_mismatch": int((sc != oc).sum()),
                   "max_rel_dist_err": float(np.max(np.abs(sd - od) /
                                                    np.maximum(np.abs(od), 1e-30)))}
            vi, vd, vc = oracle.search(view, sub, lv, pre, FINAL_NN, True, oracle.MODE_IDEAL,
                                       threads)
            gi, gd, gc = nv.search_batched(sub, lv, pre, FINAL_NN, True)
            view_ids[(lv, pre)] = gi
            ent["standalone_view"] = {
                "id_mismatch": float((gi != vi).mean()),
                "dist_bits_mismatch": float((gd.view(np.uint32) != vd.view(np.uint32)).mean()),
                "count_mismatch": int((gc != vc).sum())}
            ent["oracle_s"] = round(time.perf_counter() - t, 2)
            log(f"parity L={lv} pre={pre}: {ent}")
            out.append(ent)
    finally:
        nv.close()
    return {"path": "this rank's shard engine (search_shard + merge of its list) vs the oracle "
                    "on the shard (whole-index ties, SOAR dedupe, member-row reorder); "
                    "standalone_view: the shard renumbered as an index of its own through "
                    "search_batched vs the oracle on that view",
            "mode": "oracle ideal mode (oracle/scann_oracle.cc) vs the GPU, bit-exact ids and "
                    "distances", "points": out}, view_ids


def cpu_baseline_shard(ix, q, threads, view_ids=None):
    """The AVX2 port over this rank's shard viewed as a standalone index
    (members renumbered 0..M-1, their float rows as the dataset): the
    reference's per-rank work, timed on a bounded sample of the batch.  Its
    emulate-mode ids (FastTopNeighbors GC + the int16 truncated threshold,
    lut16_avx2.inc:432-438, 515-521) against the GPU's on the same view for
    the parity subset (SURVEY A.7's emulate-vs-ideal mismatch)."""
    from oracle import binding as oracle
    oracle.build()
    m = ix.num_members
    view = ix.standalone()
    port = oracle.Avx2Port(view)
    model, isa = cpu_info()
    sub = q[:max(threads, 250)]
    pi, _, _ = port.search(sub, LEAVES_TO_SEARCH, PRE_NN, FINAL_NN, True, threads)
    mismatch = None
    gv = (view_ids or {}).get((LEAVES_TO_SEARCH, PRE_NN))
    if gv is not None:
        mismatch = float((pi[:gv.shape[0]] != gv).mean())
    runs = []
    for _ in range(3):
        t = time.perf_counter()
        port.search(sub, LEAVES_TO_SEARCH, PRE_NN, FINAL_NN, True, threads)
        runs.append(sub.shape[0] / (time.perf_counter() - t))
    port.close()
    return dict(value=round(float(np.median(runs)), 1), unit="queries/s", cores=threads,
                kind="port", cpu_model=model, isa=isa, runs_qps=[round(x, 1) for x in runs],
                sample=f"median of 3 runs of {sub.shape[0]} queries through the AVX2 port over "
                       f"this rank's shard as a standalone index ({m} members renumbered, "
                       f"emulate-mode pipeline A), {threads} threads; no merge",
                id_mismatch_vs_gpu=mismatch,
                id_mismatch_basis=(f"the port's ids vs the GPU's search_batched on the same "
                                   f"standalone view, first {gv.shape[0]} queries (the parity "
                                   f"subset) at leaves_to_search {LEAVES_TO_SEARCH}, "
                                   f"pre_reorder_nn {PRE_NN}" if gv is not None else None))


def _peek_gpus(argv):
    """--gpus from the command line (argparse proper runs in main())."""
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    return ap.parse_known_args(argv)[0].gpus


if __name__ == "__main__":
    main()
