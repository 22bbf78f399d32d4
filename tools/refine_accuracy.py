#!/usr/bin/env python3
"""Accuracy of the fp32 tile solve against the reference's own fp32 error, per refinement threshold.

For each ALS_REFINE_MIN_PIVOT value and k, both halves of two synthetic blocks (short users / long movies) are
solved on the GPU and compared with the fp64 oracle; printed: p99 and max of the per-row norm-relative error
divided by the reference's (oracle fp32 EJML-order restatement) p99 / max on the same rows -- the ratios the
parity tests bound by 2 and 3.

  CFK_ALS_LIB=collaborative-filtering-kafka_amd/build_debug/libcfk_als.so python tools/refine_accuracy.py [thresholds...]

Thresholds below the validated 0.45 gate need the debug build (`make debug`): the product library clamps them.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    import numpy as np
    import __graft_entry__
    cfk = __graft_entry__.load_package()
    import oracle
    oracle.build()
    ths = [float(x) for x in sys.argv[1:]] or [2.0, 0.5, 0.25, 0.1, 0.05]
    lam = 0.05
    sets = []
    for n_u, n_m, nnz, seed in ((3000, 400, 90_000, 11), (2000, 150, 60_000, 3), (20000, 300, 60_000, 5)):
        ds = cfk.Dataset.synthetic_netflix(n_users=n_u, n_movies=n_m, nnz=nnz, seed=seed, nthreads=8)
        m, u, r = ds.ratings()
        sets.append((ds, oracle.build_blocks(m, u, r)))
    res = []
    for k in (32, 64, 96, 128):
        for si, (ds, b) in enumerate(sets):
            for side, rows, opp in ((0, b.movie, b.user), (1, b.user, b.movie)):
                F = np.random.default_rng(k + si).random((len(opp.ids), k))
                ref = oracle.update_side(rows, F, lam, "f64")
                ref32 = oracle.update_side(rows, F.astype(np.float32), lam, "f32")
                norm = np.linalg.norm(ref, axis=1)
                rel_ref = np.linalg.norm(ref32 - ref, axis=1) / norm
                blk = ds.shard_block(side)
                for th in ths:
                    os.environ["ALS_REFINE_MIN_PIVOT"] = str(th)
                    eng = cfk.ALSEngine(k, "f32")
                    eng.alloc_factors(1 - side, len(opp.ids))
                    eng.alloc_factors(side, blk["n_rows"])
                    eng.set_block(side, blk["row_ptr"], blk["col"], blk["ratings"], 0, len(opp.ids))
                    eng.write_factors(1 - side, F.astype(np.float32))
                    eng.solve_half(side, lam)
                    got = eng.read_factors(side)
                    eng.close()
                    rel = np.linalg.norm(got - ref, axis=1) / norm
                    d = {"k": k, "set": si, "side": side, "th": th,
                         "p99_ratio": float(np.percentile(rel, 99) / max(np.percentile(rel_ref, 99), 1e-5)),
                         "max_ratio": float(rel.max() / max(rel_ref.max(), 3.3e-5)),
                         "max_rel": float(rel.max())}
                    res.append(d)
                    print(json.dumps(d), flush=True)
    worst = {}
    for d in res:
        w = worst.setdefault(d["th"], [0.0, 0.0])
        w[0] = max(w[0], d["p99_ratio"])
        w[1] = max(w[1], d["max_ratio"])
    print(json.dumps({"worst_ratios_by_threshold (p99 bar 2, max bar 3)": worst}))


if __name__ == "__main__":
    main()
