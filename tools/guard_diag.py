#!/usr/bin/env python3
"""Diagnose non-finite results of the pre-split range guard case (tests/test_gpu_integrity.py::test_presplit_range_guard):
which rows, under which path (ALS_PRESPLIT, ALS_DUAL), for a table whose row maxima span 2^-24..scale_top."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import __graft_entry__
    import oracle
    cfk = __graft_entry__.load_package()
    ds = cfk.Dataset.synthetic_netflix(n_users=2000, n_movies=150, nnz=60_000, seed=9, nthreads=8)
    m, u, r = ds.ratings()
    b = oracle.build_blocks(m, u, r)
    for k in (64, 128):
        for top in (1.0, 2.0 ** 24):
            rng = np.random.default_rng(k + 1)
            n = len(b.user.ids)
            F = rng.random((n, k)) * 2.0 ** -rng.uniform(0, 24, size=(n, 1))
            F[0] *= top / F[0].max()
            F[1] *= 2.0 ** -24 / F[1].max()
            F = F.astype(np.float32)
            ref32 = oracle.update_side(b.movie, F, 0.05, "f32")
            for env in ({"ALS_PRESPLIT": "1"}, {"ALS_PRESPLIT": "0"}, {"ALS_PRESPLIT": "1", "ALS_DUAL": "0"},
                        {"ALS_PRESPLIT": "0", "ALS_DUAL": "0"}):
                os.environ.update(env)
                eng = cfk.ALSEngine(k, "f32")
                blk = ds.shard_block(0)
                eng.alloc_factors(1, n)
                eng.alloc_factors(0, blk["n_rows"])
                eng.set_block(0, blk["row_ptr"], blk["col"], blk["ratings"], 0, n)
                eng.write_factors(1, F)
                eng.solve_half(0, 0.05)
                got = eng.read_factors(0)
                eng.close()
                for kk in env:
                    del os.environ[kk]
                bad = np.where(~np.isfinite(got).all(axis=1))[0]
                deg = np.diff(b.movie.row_ptr)
                print(f"k={k} top={top:g} {env}: nonfinite rows {len(bad)} {bad[:8].tolist()} deg {deg[bad[:8]].tolist()} "
                      f"ref32 finite {np.isfinite(ref32).all()}", flush=True)


if __name__ == "__main__":
    main()
