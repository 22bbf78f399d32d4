#!/usr/bin/env python3
"""CPU study behind the fp16 pre-split Gram: per-row solution error of candidate Gram
splits, with the rest of the solve exact (fp64), as a multiple of the reference's OWN fp32 error (the oracle's
EJML-order fp32 restatement) on the parity tests' synthetic blocks:

  exact32  fp32 inputs, exact arithmetic (the floor any fp32 method inherits)
  bf3      three-term bf16 split, six products (hh hm mh hl lh mm): the on-the-fly path
  f16x3    two-term fp16 split of the table scaled to 2^14, three products (hh hm mh): the pre-split path
  f16x4    the same plus mm

  python tools/split_accuracy.py      (a few minutes on 8 CPUs; no GPU)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
LAM = 0.05


def split16(x, scale):
    xs = (x * scale).astype(np.float32)
    h = xs.astype(np.float16).astype(np.float32)
    m = (xs - h).astype(np.float16).astype(np.float32)
    return h.astype(np.float64), m.astype(np.float64)


def splitbf(x):
    import torch
    t = torch.from_numpy(x.astype(np.float32))
    h = t.to(torch.bfloat16).float()
    r = t - h
    m = r.to(torch.bfloat16).float()
    l = (r - m).to(torch.bfloat16).float()
    return h.double().numpy(), m.double().numpy(), l.double().numpy()


def solve_rows(side, F, mode):
    k = F.shape[1]
    out = np.zeros((len(side.row_ptr) - 1, k))
    F32 = F.astype(np.float32)
    scale = 2.0 ** (14 - int(np.ceil(np.log2(np.abs(F32).max()))))
    if mode.startswith("f16"):
        H, Mm = split16(F32, scale)
    elif mode == "bf3":
        H, Mm, L = splitbf(F32)
    for r in range(len(side.row_ptr) - 1):
        a, b = side.row_ptr[r], side.row_ptr[r + 1]
        c = side.col[a:b]
        rt = side.ratings[a:b].astype(np.float64)
        if mode == "exact32":
            Y = F32[c].astype(np.float64)
            G, rhs = Y.T @ Y, Y.T @ rt
        elif mode == "f16x3":
            h, m = H[c], Mm[c]
            G, rhs = (h.T @ h + h.T @ m + m.T @ h) / scale ** 2, (h.T @ rt + m.T @ rt) / scale
        elif mode == "f16x4":
            h, m = H[c], Mm[c]
            G, rhs = (h.T @ h + h.T @ m + m.T @ h + m.T @ m) / scale ** 2, (h.T @ rt + m.T @ rt) / scale
        else:
            h, m, l = H[c], Mm[c], L[c]
            G, rhs = h.T @ h + h.T @ m + m.T @ h + h.T @ l + l.T @ h + m.T @ m, (h + m + l).T @ rt
        G32 = G.astype(np.float32).astype(np.float64)   # the fp32 accumulator, rounded once
        out[r] = np.linalg.solve(G32 + LAM * (b - a) * np.eye(k), rhs.astype(np.float32).astype(np.float64))
    return out


def main():
    import __graft_entry__
    cfk = __graft_entry__.load_package()
    import oracle
    oracle.build()
    for k in (64, 128):
        for nu, nm, nnz, seed in ((3000, 400, 90_000, 11), (20_000, 300, 60_000, 5)):
            ds = cfk.Dataset.synthetic_netflix(n_users=nu, n_movies=nm, nnz=nnz, seed=seed, nthreads=8)
            b = oracle.build_blocks(*ds.ratings())
            for name, side, opp in (("movie", b.movie, b.user), ("user", b.user, b.movie)):
                F = np.random.default_rng(k).random((len(opp.ids), k))
                ref = oracle.update_side(side, F, LAM, "f64")
                ref32 = oracle.update_side(side, F.astype(np.float32), LAM, "f32")
                norm = np.linalg.norm(ref, axis=1)
                rr = np.linalg.norm(ref32 - ref, axis=1) / norm
                line = f"k={k} set={nu} {name}: ref32 p99 {np.percentile(rr, 99):.2e} max {rr.max():.2e}"
                for mode in ("exact32", "bf3", "f16x3", "f16x4"):
                    e = np.linalg.norm(solve_rows(side, F, mode) - ref, axis=1) / norm
                    line += (f" | {mode} p99 {np.percentile(e, 99) / np.percentile(rr, 99):.2f}x "
                             f"max {e.max() / rr.max():.2f}x")
                print(line, flush=True)


if __name__ == "__main__":
    main()
