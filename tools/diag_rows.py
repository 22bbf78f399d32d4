#!/usr/bin/env python3
"""Per-row fp32 error of the GPU solve vs the f64 oracle and vs the reference's own fp32 arithmetic
(oracle f32 = EJML LU restated), on the parity-test synthetic data. Writes gpurun_out/diag_rows.npz."""
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
    ds, b = _synthetic(cfk, om)
    res = {}
    for k in [int(x) for x in (sys.argv[1:] or ["32", "64"])]:
        rng = np.random.default_rng(k)
        for side, rows, opp in ((0, b.movie, b.user), (1, b.user, b.movie)):
            F = rng.random((len(opp.ids), k))
            ref = om.update_side(rows, F, LAM, "f64")
            r32 = om.update_side(rows, F.astype(np.float32), LAM, "f32")
            got = _one_half(cfk, side, ds.shard_block(side), F.astype(np.float32), k, "f32", len(opp.ids))
            e_got = np.linalg.norm(got - ref, axis=1) / np.linalg.norm(ref, axis=1)
            e_ref = np.linalg.norm(r32 - ref, axis=1) / np.linalg.norm(ref, axis=1)
            w = np.argsort(e_got)[::-1][:5]
            print(f"k={k} side={side} gpu max {e_got.max():.2e} p99 {np.percentile(e_got, 99):.2e} med "
                  f"{np.median(e_got):.2e} | ref32 max {e_ref.max():.2e} p99 {np.percentile(e_ref, 99):.2e} med "
                  f"{np.median(e_ref):.2e} | worst rows {list(w)} n={[int(rows.row_ptr[i + 1] - rows.row_ptr[i]) for i in w]}"
                  f" ref32 there {[f'{e_ref[i]:.1e}' for i in w]}", flush=True)
            res[f"k{k}_s{side}_gpu"] = e_got
            res[f"k{k}_s{side}_ref"] = e_ref
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez("gpurun_out/diag_rows.npz", **res)


if __name__ == "__main__":
    main()
