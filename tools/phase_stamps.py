"""Phase timeline of the front-end and select kernels (diagnostic build).

    python tools/phase_stamps.py build     (here: compiles lib/libscann_mi355x_time.so)
    python tools/phase_stamps.py [seed]    (on the GPU box)

The diagnostic library (-DSMX_PHASE_STAMPS, scann_amd/build.py build_time) writes the 100 MHz clock at phase boundaries
of topl_wave_kernel (0), seed_tau_kernel (1) and final_select_rank_kernel (2)
per query; this prints each phase's duration and where the kernels' spans go.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = os.environ.get("SMX_STAMP_LIB", os.path.join(ROOT, "scann_amd", "lib", "libscann_mi355x_time.so"))
NAMES = {0: ("topl_wave", ["load", "rounds", "compact+rank", "out+rank atomics", "lut"]),
         1: ("seed_tau", ["lut+prefix", "score loop", "k'-th select"]),
         2: ("final_select", ["load+narrow", "rank", "gid gather", "dedupe", "exact", "out"])}


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        from scann_amd import build
        print(build.build_time(force=True))
        return
    # python tools/phase_stamps.py [seed] [config]: config soar100m / deep1b
    # = rank 0's generated shard of that bench configuration as a
    # standalone index (its select at the bench's leaves_to_search / k')
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    config = sys.argv[2] if len(sys.argv) > 2 else "glove"
    os.environ["SMX_LIB"] = LIB
    path = "/tmp/smx_phase.bin"
    os.environ["SMX_PHASE_FILE"] = path
    import torch
    from bench import LEAVES_TO_SEARCH, NQ, PRE_NN, FINAL_NN, build_index
    from scann_amd import _native
    leaves, pre = LEAVES_TO_SEARCH, PRE_NN
    if config == "glove":
        db, q, ix = build_index(1_183_514, seed=2)
        nat = _native.NativeIndex(ix)
        nat.set_tuning(4096, seed, 0, 32)
    else:
        from bench import CONFIGS
        from scann_amd import generate
        cfg = CONFIGS[config]
        ds = generate.GeneratedDataset(cfg["n"], cfg["dim"], cfg["seed"],
                                       components=cfg["components"],
                                       spread=cfg.get("spread", 0.9), device=torch.device("cuda"))
        ix = generate.build_generated_shard(
            ds, cfg["leaves"], 0, cfg["split"], soar_lambda=cfg["soar"], seed=cfg["seed"],
            training_sample_size=cfg["train_sample"],
            training_iterations=cfg.get("train_iterations", 8), counts_from_all_ranks=False)
        q = ds.queries(NQ, cfg["seed"] + 1000)
        leaves = cfg["leaves_to_search"]
        nat = _native.NativeIndex(ix.standalone())
        nat.set_tuning(0, seed)
    qd = torch.from_numpy(q).cuda()
    oi = torch.zeros((NQ, FINAL_NN), dtype=torch.int32, device="cuda")
    od = torch.zeros((NQ, FINAL_NN), dtype=torch.float32, device="cuda")
    for _ in range(4):
        nat.search_batched_device(qd.data_ptr(), NQ, leaves, pre, FINAL_NN, True,
                                  oi.data_ptr(), od.data_ptr(), None)
    torch.cuda.synchronize()
    full = np.fromfile(path, dtype=np.uint64).reshape(3, 4096, 8).astype(np.int64)
    r = full[:, :NQ]
    wl0 = full[1, 4095, :3]   # the fused work list's block 0: start, leaf_item0 written, end
    if (wl0 > 0).all():
        t0 = r[1][(r[1][:, 0] > 0), 0].min()
        print("work-list block 0 (us from the first seed block's start): start %.1f, "
              "leaf_item0 written %.1f, end %.1f" % tuple((wl0 - t0) / 100.0))
    for kid, (name, phases) in NAMES.items():
        t = r[kid]
        n = len(phases) + 1
        ok = (t[:, :n] > 0).all(1)
        t = t[ok][:, :n]
        if not len(t):
            print(f"{name}: no stamps")
            continue
        t0 = t[:, 0].min()
        span = (t[:, n - 1].max() - t0) / 100.0
        st = (t[:, 0] - t0) / 100.0
        en = (t[:, n - 1] - t0) / 100.0
        print(f"{name}: {len(t)} queries, span {span:.1f} us; start p50 {np.median(st):.1f} "
              f"max {st.max():.1f}; end p10 {np.percentile(en, 10):.1f} p50 {np.median(en):.1f} "
              f"max {en.max():.1f}")
        for i, ph in enumerate(phases):
            d = (t[:, i + 1] - t[:, i]) / 100.0
            print(f"    {ph:18s} p50 {np.median(d):6.2f} p90 {np.percentile(d, 90):6.2f} "
                  f"max {d.max():6.2f} us")


if __name__ == "__main__":
    main()
