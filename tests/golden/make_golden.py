"""Generate the committed golden fixtures (run HERE, in the build container; never on the GPU box).

  python tests/golden/make_golden.py

Inputs: the reference's own data files (copied verbatim as fixtures: data_sample_tiny.txt,
data_sample_medium.txt from /root/reference/data/), the CPU oracle (oracle/), and the reference's
scripts/calculate_mse.py, which is executed as a subprocess on an oracle-written prediction CSV to pin the
CSV layout + MSE definition (scripts/calculate_mse.py:60-90). Nothing from the reference is copied except
those data files; the reference script is only run, never stored.

Outputs:
  tiny_k10_n10_p4_seed42_f64.npz     U_N, M_{N-1} (ascending ids), MSE          (BASELINE configs[0] shape)
  medium_k10_n10_p4_seed42_f64.npz   same for the medium sample                 (BASELINE configs[1])
  known_answers.json                 exact-rational solutions of small systems  (pins the update formula)
  tiny_k5_n7_seed42_mse_reference.json  MSE printed by the reference's calculate_mse.py on the oracle's CSV
  tiny_k5_n7_seed42_prediction.csv.gz   that CSV (oracle writer, Java Double.toString layout)
"""
from __future__ import annotations

import gzip
import json
import os
import random
import re
import subprocess
import sys
import tempfile
from fractions import Fraction

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

REFERENCE_MSE_SCRIPT = "/root/reference/scripts/calculate_mse.py"


def als_golden(name: str, k: int, n: int, seed: int, lam: float = 0.05, parts: int = 4):
    path = os.path.join(HERE, f"data_sample_{name}.txt")
    m, u, r = oracle.parse_netflix(path)
    blocks = oracle.build_blocks(m, u, r, parts)
    U, M = oracle.run_als(blocks, k, lam, n, seed=seed, precision="f64")
    mse = oracle.mse(blocks, U, M)
    out = os.path.join(HERE, f"{name}_k{k}_n{n}_p{parts}_seed{seed}_f64.npz")
    np.savez_compressed(out, U=U, M=M, mse=np.float64(mse), user_ids=blocks.user.ids, movie_ids=blocks.movie.ids,
                        k=k, n=n, seed=seed, lam=np.float32(lam))
    print(f"{out}: mse={mse:.12f}")


def solve_exact(Y, r, lam_f32: float):
    """(Y^T Y + lambda * n * I) x = Y^T r in exact rational arithmetic (Gauss-Jordan)."""
    n = len(Y)
    k = len(Y[0])
    lam = Fraction(lam_f32)
    A = [[sum(Fraction(Y[t][i]) * Fraction(Y[t][j]) for t in range(n)) for j in range(k)] for i in range(k)]
    for i in range(k):
        A[i][i] += lam * n
    b = [sum(Fraction(Y[t][i]) * r[t] for t in range(n)) for i in range(k)]
    M = [row[:] + [b[i]] for i, row in enumerate(A)]
    for c in range(k):
        p = next(i for i in range(c, k) if M[i][c] != 0)
        M[c], M[p] = M[p], M[c]
        inv = 1 / M[c][c]
        M[c] = [v * inv for v in M[c]]
        for i in range(k):
            if i != c and M[i][c] != 0:
                f = M[i][c]
                M[i] = [a - f * b for a, b in zip(M[i], M[c])]
    return [M[i][k] for i in range(k)]


def known_answers():
    rnd = random.Random(20191205)
    cases = []
    for n, k in [(1, 1), (1, 2), (2, 2), (3, 2), (2, 3), (3, 4), (5, 4), (1, 5), (7, 3), (4, 10)]:
        # factor values exactly representable in float32 (k/8 steps), ratings 1..5
        Y = [[rnd.randint(0, 16) / 8.0 for _ in range(k)] for _ in range(n)]
        r = [rnd.randint(1, 5) for _ in range(n)]
        lam = float(np.float32(0.05))
        x = solve_exact(Y, r, lam)
        cases.append({"n": n, "k": k, "Y": Y, "r": r, "lambda": "0.05",
                      "x": [float(v) for v in x], "x_exact": [f"{v.numerator}/{v.denominator}" for v in x]})
    out = os.path.join(HERE, "known_answers.json")
    with open(out, "w") as f:
        json.dump(cases, f, indent=1)
    print(f"{out}: {len(cases)} systems")


def reference_mse_fixture():
    path = os.path.join(HERE, "data_sample_tiny.txt")
    m, u, r = oracle.parse_netflix(path)
    blocks = oracle.build_blocks(m, u, r, 4)
    U, M = oracle.run_als(blocks, 5, 0.05, 7, seed=42, precision="f64")
    P = oracle.prediction_matrix(U, M)
    with tempfile.TemporaryDirectory() as td:
        csv = os.path.join(td, "prediction_matrix")
        oracle.save_dense_csv(P, csv)
        res = subprocess.run([sys.executable, REFERENCE_MSE_SCRIPT, path, csv], check=True, capture_output=True,
                             text=True)
        mse = float(re.search(r"MSE:\s*([0-9.eE+-]+)", res.stdout).group(1))
        with open(csv, "rb") as f, gzip.open(os.path.join(HERE, "tiny_k5_n7_seed42_prediction.csv.gz"), "wb") as g:
            g.write(f.read())
    out = os.path.join(HERE, "tiny_k5_n7_seed42_mse_reference.json")
    with open(out, "w") as f:
        json.dump({"ratings": "data_sample_tiny.txt", "k": 5, "iterations": 7, "lambda": "0.05", "seed": 42,
                   "precision": "f64 oracle, fp32 prediction matrix", "reference_script": "scripts/calculate_mse.py",
                   "stdout": res.stdout, "mse": mse}, f, indent=1)
    print(f"{out}: reference calculate_mse.py MSE={mse!r}")


if __name__ == "__main__":
    oracle.build()
    als_golden("tiny", 10, 10, 42)
    als_golden("medium", 10, 10, 42)
    known_answers()
    reference_mse_fixture()
