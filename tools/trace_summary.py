#!/usr/bin/env python3
"""Per-launch-shape summary of a rocprofv3 kernel trace: the ALS solve kernel's main (FULL + PARTIAL) launch
of each half vs its REDUCE launch, told apart by grid size (the movie and user main launches are the two
largest grids). The rocprofv3 --stats CSV averages all launches of one template together; this splits them
so the averages can be compared with bench.py's roofline.avg_launch_ms.

  python tools/trace_summary.py profiles/<dir>/kernel_trace.csv > profiles/<dir>/main_launch_summary.json
"""
import csv
import json
import sys
from collections import defaultdict


def main(path):
    d = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if "als_solve" not in r["Kernel_Name"]:
            continue
        d[(r["Kernel_Name"], int(r.get("Grid_Size") or r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    rows = sorted(d.items(), key=lambda kv: -kv[0][1])
    out = {"source": path, "launches": []}
    for i, ((name, grid), ms) in enumerate(rows):
        role = {0: "user main", 1: "movie main"}.get(i, "reduce")
        out["launches"].append({"kernel": name.split("(")[0], "grid": grid, "role": role, "calls": len(ms),
                                "avg_ms": sum(ms) / len(ms), "min_ms": min(ms), "max_ms": max(ms)})
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
