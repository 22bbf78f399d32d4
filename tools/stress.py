#!/usr/bin/env python3
"""Repeat-solve stress test for transient kernel faults on the full Netflix-shape workload.

Solves the movie half (fixed U0) and the user half (fixed M) R times each with identical inputs and reports,
for every repetition, the rows that differ from the row-wise majority result, with their error against an fp64
restatement of the update (MFeatureCalculator.java:82-99). A correct kernel gives 0 everywhere.

  STRESS_REPS=40 python tools/stress.py [VAR=VAL[,VAR=VAL]] ...       (variants = env at engine creation)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import __graft_entry__
    cfk = __graft_entry__.load_package()
    reps = int(os.environ.get("STRESS_REPS", "40"))
    k = 64
    lam = 0.05
    ds = cfk.Dataset.synthetic_netflix(480_189, 17_770, 100_000_000, 0xA15, nthreads=16)
    U0 = ds.init_user_factors(k, 42)
    blocks = [ds.shard_block(0), ds.shard_block(1)]

    def fp64_err(side, i, x, opp):
        b = blocks[side]
        cols = b["col"][b["row_ptr"][i]:b["row_ptr"][i + 1]]
        Y = opp[cols, :k].astype(np.float64)
        r = b["ratings"][b["row_ptr"][i]:b["row_ptr"][i + 1]].astype(np.float64)
        A = Y.T @ Y + np.float64(np.float32(lam)) * len(cols) * np.eye(k)
        ref = np.linalg.solve(A, Y.T @ r)
        return float(np.max(np.abs(x[:k] - ref)) / np.max(np.abs(ref)))

    summary = {}
    for v in (sys.argv[1:] or ["DEFAULT=1"]):
        saved = dict(os.environ)
        for kv in v.split(","):
            a, c = kv.split("=")
            os.environ[a] = c
        eng = cfk.ALSEngine(k, "f32")
        eng.use_torch_stream()
        for side in (0, 1):
            b = ds.shard_coo(side)
            eng.alloc_factors(side, b["n_slots"])
            eng.set_block_coo(side, b["n_rows"], b["rows"], b["cols"], b["ratings"], 0, ds.shard_info(1 - side)["n_slots"])
        os.environ.clear()
        os.environ.update(saved)
        eng.write_factors(1, U0)
        eng.solve_half(0, lam)
        M0 = eng.read_factors(0)
        res = {}
        for side, opp in ((0, U0), (1, M0)):
            outs = []
            for rep in range(reps):
                eng.write_factors(1 - side, opp)
                eng.solve_half(side, lam)
                outs.append(eng.read_factors(side))
            stack = np.stack(outs)
            # row-wise majority: a row equal to the result of most repetitions
            ref = stack[0].copy()
            for i in np.nonzero(np.any(stack != stack[0][None], axis=2).any(axis=0))[0]:
                vals, counts = np.unique(stack[:, i, :], axis=0, return_counts=True)
                ref[i] = vals[np.argmax(counts)]
            bad = []
            for rep in range(reps):
                rows = np.nonzero(np.any(stack[rep] != ref, axis=1))[0]
                for i in rows[:4]:
                    bad.append({"rep": rep, "row": int(i), "deg": int(blocks[side]["row_ptr"][i + 1] - blocks[side]["row_ptr"][i]),
                                "err_bad": fp64_err(side, i, stack[rep][i], opp), "err_ref": fp64_err(side, i, ref[i], opp)})
                if len(rows):
                    print(f"{v} side {side} rep {rep}: {len(rows)} rows differ from the majority", flush=True)
            res[["movie", "user"][side]] = {"reps": reps, "bad_reps": len({b["rep"] for b in bad}),
                                            "bad_rows": sum(1 for _ in bad), "samples": bad[:8]}
            print(v, ["movie", "user"][side], json.dumps(res[["movie", "user"][side]]), flush=True)
            del stack, outs
        summary[v] = res
        eng.close()
    print(json.dumps({"stress": summary}))


if __name__ == "__main__":
    main()
