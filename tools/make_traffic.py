#!/usr/bin/env python3
"""profiles/<dir>/pmc_fetch_size.csv + pmc_write_size.csv -> profiles/traffic.json (read by bench.py).

HBM-side bytes per launch of the main solve kernel (the FULL+PARTIAL launch of each half), averaged over the
movie- and user-half launches like bench.py's roofline.achieved. Corrections per MI355X_MICROARCH.md §HBM:
FETCH_SIZE / WRITE_SIZE are in KiB; FETCH_SIZE is doubled (gfx950 tallies 128-B requests as 64 B for wide
streaming reads -- our gathers are 16 B/lane pieces of 256-B rows, an uncalibrated width, so treat the read
side as an estimate); WRITE_SIZE is taken as is. Infinity-Cache hits are counted by these counters.
"""
import csv
import json
import sys
from collections import defaultdict


def per_dispatch(path, counter):
    out = defaultdict(float)
    grid = {}
    for r in csv.DictReader(open(path)):
        if "als_solve_" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            out[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
            grid[int(r["Dispatch_Id"])] = int(r["Grid_Size"])
    return out, grid


def main(d, k=64, nnz=100_000_000):
    fetch, grid = per_dispatch(f"{d}/pmc_fetch_size.csv", "FETCH_SIZE")
    write, grid_w = per_dispatch(f"{d}/pmc_write_size.csv", "WRITE_SIZE")
    # main launches = the two largest grids (movie: FULL+PARTIAL chunks, user: one task per user)
    sizes = sorted(set(grid.values()), reverse=True)[:2]
    res = {}
    for g in sizes:
        f = [v for k_, v in fetch.items() if grid[k_] == g]
        w = [v for k_, v in write.items() if grid_w.get(k_) == g]
        res[g] = (sum(f) / len(f) * 2 * 1024, sum(w) / len(w) * 1024)
    per_launch = sum(fb + wb for fb, wb in res.values()) / len(res)
    out = {"k": k, "nnz": nnz, "hbm_bytes_per_launch": per_launch,
           "per_grid": {str(g): {"fetch_bytes_x2": fb, "write_bytes": wb} for g, (fb, wb) in res.items()},
           "source": d, "note": "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, KiB->B; MALL hits included"}
    json.dump(out, open("profiles/traffic.json", "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1])
