#!/usr/bin/env python3
"""What goes wrong in a nondeterministic split row (PARTIAL slot) of the Netflix-shape movie half.

Repeats {write U0, movie half, copy partial slots} REPS times with a fixed launch generation (slots bitwise
comparable), finds slots that differ from the majority, decodes them (SlotCodec, als_kernels.hip) into the
64 x 64 Gram + RHS they hold, and explains the difference D = G_bad - G_good:
  - which accumulator tiles / RHS words differ,
  - the rank of D,
  - whether D is (+/-) the contribution of one or two 32-entry blocks of the chunk (a dropped or doubled block),
  - the per-block best fit otherwise.

  REPS=10 [READ_U=1] python tools/split_diag.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

M32 = 0xFFFFFFFF
STEP = 0x632BE5AB
C = 4
NT = C * (C + 1) // 2
NWORDS = NT * 4 + C
SW = NWORDS + 1


def mix32(x):
    import numpy as np
    x = x.astype(np.uint64) & M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & M32
    x ^= x >> np.uint64(16)
    return x & M32


def decode(words, slot, gen=1):
    """words: [SW * 64] uint32 of one slot ([word][lane]) -> float32 plain words [NWORDS][64], check ok?"""
    import numpy as np
    lanes = np.arange(64, dtype=np.uint64)
    key = mix32((np.uint64(gen) * np.uint64(0x9E3779B1) & M32) ^ mix32(np.uint64(slot) * np.uint64(64) + lanes))
    w = words.reshape(SW, 64).astype(np.uint64)
    plain = np.zeros((NWORDS, 64), np.uint64)
    for i in range(NWORDS):
        plain[i] = w[i] ^ ((key + np.uint64(i * STEP)) & M32)
    chk = (plain.sum(axis=0) & M32) == (w[NWORDS] ^ ((key + np.uint64(NWORDS * STEP)) & M32))
    return plain.astype(np.uint32).view(np.float32), bool(chk.all())


def gram_of(plain):
    """Accumulator layout (als_kernels.hip, C = 4): tile p = (b1 <= b2), lane (g, c), reg r holds
    G[4 * (4g + r) + b1][4c + b2]; RHS word NT*4 + b of lane (g, c) is the group-g part of feature 4c + b."""
    import numpy as np
    G = np.zeros((64, 64))
    rhs = np.zeros(64)
    p = 0
    for b1 in range(C):
        for b2 in range(b1, C):
            for r in range(4):
                for lane in range(64):
                    g, c = lane >> 4, lane & 15
                    f1, f2 = 4 * (4 * g + r) + b1, 4 * c + b2
                    v = float(plain[p * 4 + r, lane])
                    G[f1, f2] = v
                    G[f2, f1] = v
            p += 1
    for b in range(C):
        for lane in range(64):
            rhs[4 * (lane & 15) + b] += float(plain[NT * 4 + b, lane])
    return G, rhs


def main():
    import numpy as np
    import __graft_entry__
    cfk = __graft_entry__.load_package()
    os.environ["ALS_DEBUG_FIXED_GEN"] = "1"
    reps = int(os.environ.get("REPS", "10"))
    read_u = os.environ.get("READ_U", "0") == "1"
    lam = 0.05
    ds = cfk.Dataset.synthetic_netflix(480_189, 17_770, 100_000_000, 0xA15, nthreads=16)
    U0 = ds.init_user_factors(64, 42)
    eng = cfk.ALSEngine(64, "f32")
    for side in (0, 1):
        b = ds.shard_coo(side)
        eng.alloc_factors(side, b["n_slots"])
        eng.set_block_coo(side, b["n_rows"], b["rows"], b["cols"], b["ratings"], 0, ds.shard_info(1 - side)["n_slots"])
    # partial slots and movie factors of every rep are compared with rep 0's on the fly (bounded memory)
    blk = ds.shard_block(0)
    deg = np.diff(blk["row_ptr"])
    nnz_padded = eng.block_stats(0)["nnz_padded"]
    chunk = min(max(nnz_padded // 4096, 1024), 32768)
    chunk = (chunk + 31) // 32 * 32
    owner = []                                  # slot -> (row, chunk index)
    for i, d in enumerate(deg):
        if d > chunk:
            for c in range(-(-int(d) // chunk)):
                owner.append((i, c))
    n_slots = len(owner)
    P0 = M0 = None
    diffs = {}                                  # slot -> {rep: words}
    movie_rows = set()
    for rep in range(reps):
        eng.write_factors(1, U0)
        eng.solve_half(0, lam)
        M = eng.read_factors(0)
        P = eng.debug_partials()[:n_slots * SW * 64].reshape(n_slots, SW * 64)
        if P0 is None:
            P0, M0 = P, M
        else:
            for s in np.nonzero(np.any(P != P0, axis=1))[0]:
                diffs.setdefault(int(s), {})[rep] = P[s].copy()
            movie_rows |= set(np.nonzero(np.any(M != M0, axis=1))[0].tolist())
        eng.solve_half(1, lam)
        if read_u:
            eng.read_factors(1)       # the determinism test's sequence: U read back before U0 is rewritten
        eng.synchronize()
        if rep % 25 == 0:
            print(f"rep {rep} done", flush=True)
    eng.close()
    out = {"reps": reps, "chunk": chunk, "n_slots": n_slots, "bad": []}
    for s, reps_d in sorted(diffs.items()):
        if len(reps_d) > reps // 2:             # rep 0 was the odd one out
            good, bad_list = next(iter(reps_d.values())), [(0, P0[s])]
        else:
            good, bad_list = P0[s], list(reps_d.items())
        for rep, words in bad_list:
            row, c = owner[s]
            pg, okg = decode(good, s)
            pb, okb = decode(words, s)
            diff_words = np.nonzero(np.any(pg != pb, axis=1))[0].tolist()
            Gg, rg = gram_of(pg)
            Gb, rb = gram_of(pb)
            D = Gb - Gg
            ev = np.linalg.eigvalsh(D)
            rank = int(np.sum(np.abs(ev) > 1e-4 * max(1e-30, np.abs(ev).max())))
            # per 32-entry block contributions of the chunk (logical entry order = CSR order)
            lo = int(blk["row_ptr"][row]) + c * chunk
            hi = min(int(blk["row_ptr"][row + 1]), lo + chunk)
            Y = U0[blk["col"][lo:hi], :64].astype(np.float64)
            R = blk["ratings"][lo:hi].astype(np.float64)
            fits = []
            for b0 in range(0, hi - lo, 32):
                Gb_ = Y[b0:b0 + 32].T @ Y[b0:b0 + 32]
                rb_ = Y[b0:b0 + 32].T @ R[b0:b0 + 32]
                for sgn in (-1.0, 1.0):
                    res = np.linalg.norm(D - sgn * Gb_) / max(1e-300, np.linalg.norm(D))
                    fits.append((res, b0 // 32, sgn, float(np.linalg.norm((rb - rg) - sgn * rb_) / max(1e-30, np.linalg.norm(rb - rg)))))
            fits.sort()
            Gfull = Y.T @ Y
            # RHS words: lane (g, j), word NT*4 + b = sum over entries e = 4t + g of each 32-entry block of
            # r_e * y_e[4j + b]. Explain each differing lane by one entry (a dropped/doubled FMA) or one block.
            lane_info = []
            for w in diff_words:
                if w < NT * 4:
                    continue
                bcomp = w - NT * 4
                for lane in np.nonzero(pg[w] != pb[w])[0]:
                    g, j = lane >> 4, lane & 15
                    d = float(pb[w, lane]) - float(pg[w, lane])
                    f = 4 * j + bcomp
                    ent = np.arange(g, hi - lo, 4)            # logical entries of group g
                    contrib = R[ent] * Y[ent, f]
                    best = int(np.argmin(np.abs(np.abs(contrib) - abs(d)))) if len(ent) else -1
                    blocks = np.add.reduceat(contrib, np.arange(0, len(contrib), 8)) if len(contrib) else []
                    bb = int(np.argmin(np.abs(np.abs(blocks) - abs(d)))) if len(blocks) else -1
                    lane_info.append({"word": int(w), "lane": int(lane), "diff": d, "good": float(pg[w, lane]),
                                      "best_entry": int(ent[best]) if best >= 0 else None,
                                      "entry_contrib": float(contrib[best]) if best >= 0 else None,
                                      "best_block": bb, "block_contrib": float(blocks[bb]) if bb >= 0 else None})
            out["bad"].append({
                "slot": s, "row": row, "chunk_index": c, "deg": int(deg[row]), "rep": rep, "check_ok": [okg, okb],
                "n_differing_words": len(diff_words), "differing_words": diff_words[:48],
                "tiles_differing": sorted({w // 4 for w in diff_words if w < NT * 4}),
                "rhs_differs": any(w >= NT * 4 for w in diff_words),
                "D_norm_rel": float(np.linalg.norm(D) / np.linalg.norm(Gg)),
                "good_vs_fp64_chunk_gram_rel": float(np.linalg.norm(Gg - Gfull) / np.linalg.norm(Gfull)),
                "D_rank": rank, "D_eig_min_max": [float(ev.min()), float(ev.max())],
                "rhs_diff_rel": float(np.linalg.norm(rb - rg) / np.linalg.norm(rg)),
                "best_block_fits": [{"resid": float(f[0]), "block": f[1], "sign": f[2], "rhs_resid": f[3]} for f in fits[:3]],
                "chunk_blocks": (hi - lo + 31) // 32,
                "rhs_lanes": lane_info[:64],
            })
            print(json.dumps(out["bad"][-1]), flush=True)
    out["movie_rows_differing"] = len(movie_rows)
    print(json.dumps({"split_diag": {k: v for k, v in out.items() if k != "bad"}, "n_bad": len(out["bad"])}))


if __name__ == "__main__":
    main()
