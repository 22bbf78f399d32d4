import os, sys
import numpy as np
ROOT = "/root/repo"
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import __graft_entry__
from oracle import oracle as om
from test_gpu_parity import _synthetic, _one_half, LAM
cfk = __graft_entry__.load_package()
k = 64
ds, b = _synthetic(cfk, om)
for side, rows, opp in ((0, b.movie, b.user), (1, b.user, b.movie)):
    F = np.random.default_rng(k).random((len(opp.ids), k)).astype(np.float32)
    outs = {}
    for v in ("ALS_MFMA_WAVES=2,ALS_DEBUG_SKIP_SOLVE=1", "ALS_MFMA_WAVES=3,ALS_DEBUG_SKIP_SOLVE=1",
              "ALS_MFMA_WAVES=2,ALS_DEBUG_SKIP_REFINE=1", "ALS_MFMA_WAVES=3,ALS_DEBUG_SKIP_REFINE=1"):
        saved = dict(os.environ)
        for kv in v.split(","):
            a, c = kv.split("="); os.environ[a] = c
        outs[v] = _one_half(cfk, side, ds.shard_block(side), F, k, "f32", len(opp.ids))
        os.environ.clear(); os.environ.update(saved)
    ks = list(outs)
    for i in (0, 2):
        a, c = outs[ks[i]], outs[ks[i + 1]]
        d = np.abs(a - c).max(axis=1)
        print(side, ks[i], "vs 3-wave: rows differing", int((d > 1e-3 * np.abs(a).max(axis=1)).sum()), "/", len(d), "max", d.max(), flush=True)
