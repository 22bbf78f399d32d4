#!/usr/bin/env python3
"""Compare kernel variants (env settings) on one half against the f64 oracle: per-row norm-relative error.
  python tools/diag_variants.py [k]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch  # noqa: F401
    import __graft_entry__
    from oracle import oracle as om
    from test_gpu_parity import _synthetic, _one_half, LAM
    cfk = __graft_entry__.load_package()
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    ds, b = _synthetic(cfk, om)
    for side, rows, opp in ((0, b.movie, b.user), (1, b.user, b.movie)):
        F = np.random.default_rng(k).random((len(opp.ids), k))
        ref = om.update_side(rows, F, LAM, "f64")
        for v in ("ALS_MFMA_WAVES=2", "ALS_MFMA_WAVES=3", "ALS_GRAM=f32", "ALS_GRAM=f32,ALS_MFMA_WAVES=3",
                  "ALS_MFMA_WAVES=3,ALS_CHUNK=100000", "ALS_MFMA_WAVES=2,ALS_CHUNK=100000"):
            saved = dict(os.environ)
            for kv in v.split(","):
                a, c = kv.split("=")
                os.environ[a] = c
            got = _one_half(cfk, side, ds.shard_block(side), F.astype(np.float32), k, "f32", len(opp.ids))
            os.environ.clear()
            os.environ.update(saved)
            rel = np.linalg.norm(got - ref, axis=1) / np.linalg.norm(ref, axis=1)
            print(f"side={side} k={k} {v:40s} p50={np.median(rel):.2e} max={rel.max():.2e} bad_rows={(rel > 1e-3).sum()}/{len(rel)}", flush=True)


if __name__ == "__main__":
    main()
