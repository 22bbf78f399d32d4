"""Fault injection for tests/test_gpu_integrity.py, run in a child process against the DEBUG build.

The injection knob (ALS_DEBUG_REDUCE_GEN_SKEW: the REDUCE launch decodes with another launch's generation) exists only
in collaborative-filtering-kafka_amd/build_debug/libcfk_als.so (CFK_DEBUG_KNOBS); the product library has no such
knob, so the child selects the debug build with CFK_ALS_LIB before the package loads it. Prints one JSON line per case.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    import numpy as np
    import torch  # noqa: F401
    import __graft_entry__
    cfk = __graft_entry__.load_package()
    from cfk_amd._lib import ALSError, LIB_PATH
    assert "build_debug" in LIB_PATH, LIB_PATH
    import oracle
    ds = cfk.Dataset.synthetic_netflix(n_users=2000, n_movies=150, nnz=60_000, seed=3, nthreads=8)
    m, u, r = ds.ratings()
    b = oracle.build_blocks(m, u, r)
    blk = ds.shard_block(0)
    for k, prec in ((64, "f32"), (128, "f32"), (32, "f32"), (10, "f64")):
        F = np.random.default_rng(2).random((len(b.user.ids), k)).astype(np.float32 if prec == "f32" else np.float64)
        eng = cfk.ALSEngine(k, prec)
        eng.alloc_factors(1, len(b.user.ids))
        eng.alloc_factors(0, blk["n_rows"])
        eng.set_block(0, blk["row_ptr"], blk["col"], blk["ratings"], 0, len(b.user.ids))
        eng.write_factors(1, F)
        st = eng.block_stats(0)
        eng.solve_half(0, 0.05)
        raised = None
        try:
            eng.read_factors(0)
        except ALSError as ex:
            raised = str(ex)
        rec = eng.integrity_status(reset=True)
        after = eng.integrity_status()
        eng.read_factors(0)   # cleared: synchronising calls succeed again
        eng.close()
        print(json.dumps({"k": k, "prec": prec, "raised": raised, "rec": rec, "after": after, "stats": st,
                          "n_movies": len(b.movie.ids)}), flush=True)


if __name__ == "__main__":
    main()
