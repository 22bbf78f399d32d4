#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (gpurun_out/pmc_<tag>_*/run_counter_collection.csv) per kernel dispatch
of the ALS solve kernels: one row per dispatch (grid size distinguishes movie / user / reduce launches)."""
import csv
import glob
import sys
from collections import defaultdict

tag = sys.argv[1] if len(sys.argv) > 1 else "a"
rows = defaultdict(dict)   # (kernel, grid, dispatch order within kernel) -> counters
for f in sorted(glob.glob(f"gpurun_out/pmc_{tag}_*/run_counter_collection.csv")):
    seen = defaultdict(int)
    last_disp = {}
    for r in csv.DictReader(open(f)):
        if "als_" not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"].split("::")[-1].split("(")[0]
        key0 = (name, int(r["Grid_Size"]))
        d = r["Dispatch_Id"]
        if last_disp.get(key0) != d:
            seen[key0] += 1
            last_disp[key0] = d
        key = key0 + (seen[key0],)
        rows[key][r["Counter_Name"]] = float(r["Counter_Value"])
        rows[key]["dur_ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
for key in sorted(rows):
    c = rows[key]
    print(key, " ".join(f"{k}={v:.4g}" for k, v in sorted(c.items())))
