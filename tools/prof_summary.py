#!/usr/bin/env python3
"""gpurun_out/prof_<tag>/ (tools/profile_round.sh) -> profiles/<name>/ summaries + profiles/traffic.json.

Writes:
  kernel_stats.csv            rocprofv3 --stats of the 20-step bench run (as produced)
  main_launch_summary.json    per half (movie / user main launch, reduce launch): calls, avg/min/max ms from the
                              kernel trace -- the figure bench.py's HIP-event avg_launch_ms must agree with
  pmc_summary.json            per half: FETCH_SIZE x2 + WRITE_SIZE bytes per launch (MI355X guide corrections:
                              KiB -> B, FETCH doubled on gfx950), and the SQ counters of the full launch and of
                              the Gram alone (ALS_DEBUG_SKIP_SOLVE=1): MFMA busy share, issue stalls, clock
  bench_line.json             the bench.py line of the same call
and profiles/counters_k<k>.json (read by bench.py, which uses it only when its lib_sha256 -- the library the profiled
bench line reports -- is the library it runs): per side the HBM bytes per launch, the MFMA-pipe busy share of
the whole launch and of the Gram alone (debug build, ALS_DEBUG_SKIP_SOLVE=1), the sustained clock, and the solve
phase = whole launch minus Gram-only counters (its share of the launch's cycles, MFMA busy and VALU issue share).
Sides: the main solve kernel dispatch with the largest grid is the user half (480,189 tasks), the next the movie
half (FULL + PARTIAL tasks); the REDUCE kernel instantiation is recognised by its last template argument.

  python tools/prof_summary.py <tag> <profiles subdir> [<movie launches per half> <user launches per half>]
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def mfma_args(name):
    """template arguments of an als_solve_mfma instantiation: <KP, MINW, SPLIT, PRESPLIT, REDUCE, GRIDLOOP>
    (als_kernels.hip)"""
    if "als_solve_mfma<" not in name:
        return None
    return [a.strip() for a in name.split("als_solve_mfma<", 1)[1].split(">")[0].split(",")]


def is_reduce(name):
    a = mfma_args(name)
    return bool(a) and len(a) > 4 and a[4] == "true"


def is_fallback(name):
    """the pre-split range guard's grid-stride fallback launch (waves exit at once while the table is in range)"""
    a = mfma_args(name)
    return bool(a) and len(a) > 5 and a[5] == "true"


def role_of(name, grid, grids):
    if "als_solve" not in name:
        return None
    if "als_solve_dual" in name:
        return "dual"
    if is_reduce(name):
        return "reduce"
    if is_fallback(name):
        return "fallback"
    big = sorted(grids, reverse=True)
    if grid == big[0]:
        return "user"
    if len(big) > 1 and grid == big[1]:
        return "movie"
    return "other"


def half_groups(rows, per_half):
    """{Dispatch_Id: (role, half index)} for the main launches (als_solve_mfma, neither REDUCE nor the guard's
    fallback) of the rows, in dispatch order: every iteration runs per_half["movie"] movie-half launches (one per slot
    chunk), then per_half["user"] user-half launches (bench.py config launches_per_half). None when the launch count
    does not fit that pattern (the caller then tells the halves apart by grid size)."""
    if not per_half:
        return None
    lm, lu = int(per_half["movie"]), int(per_half["user"])
    ids = sorted({int(r["Dispatch_Id"]) for r in rows if "als_solve_mfma" in r["Kernel_Name"]
                  and not is_reduce(r["Kernel_Name"]) and not is_fallback(r["Kernel_Name"])})
    if not ids or len(ids) % (lm + lu):
        return None
    out = {}
    for i, d in enumerate(ids):
        pos = i % (lm + lu)
        out[d] = ("movie" if pos < lm else "user", i // (lm + lu))
    return out


def counters_name(k, cfg):
    """profiles/ file of a profiled configuration (bench.py counters_path reads the same name): counters_k<k>.json for
    the metric's workload on the whole dataset, counters_k<k>_<workload>[_shard<G>].json otherwise"""
    wl = cfg.get("workload_name", "netflix")
    shard = cfg.get("shard_of")
    if wl == "netflix" and not shard:
        return f"counters_k{k}.json"
    return f"counters_k{k}_{wl}" + (f"_shard{shard}" if shard else "") + ".json"


def load_rows(pattern):
    rows = []
    for f in glob.glob(pattern, recursive=True):
        rows += list(csv.DictReader(open(f)))
    return rows


def main(tag, name, launches=None):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles", name)
    os.makedirs(dst, exist_ok=True)
    out = {}
    # --- kernel trace ---
    tr = load_rows(f"{src}/trace/**/*kernel_trace.csv")
    st = glob.glob(f"{src}/trace/**/*kernel_stats.csv", recursive=True)
    if st:
        shutil.copy(st[0], os.path.join(dst, "kernel_stats.csv"))
    bl = os.path.join(src, "bench.json")
    cfg0 = {}
    if os.path.exists(bl):
        ls = [l for l in open(bl) if l.startswith("{")]
        cfg0 = json.loads(ls[-1]).get("config", {}) if ls else {}
    per_half = cfg0.get("launches_per_half") or launches

    grid = lambda r: int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
    grids = {grid(r) for r in tr if "als_solve_mfma" in r["Kernel_Name"] and not is_reduce(r["Kernel_Name"])
             and not is_fallback(r["Kernel_Name"])}
    groups = half_groups(tr, per_half)
    dur = defaultdict(list)
    half_ms = defaultdict(lambda: defaultdict(float))   # one half = the sum of its chunk launches
    for r in tr:
        ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        g = groups.get(int(r["Dispatch_Id"])) if groups else None
        if g:
            half_ms[g[0]][g[1]] += ms
            continue
        role = role_of(r["Kernel_Name"], grid(r), grids)
        if role:
            dur[role].append(ms)
    for role, h in half_ms.items():
        dur[role] = [h[i] for i in sorted(h)]
    out["trace"] = {k: {"calls": len(v), "avg_ms": sum(v) / len(v), "min_ms": min(v), "max_ms": max(v),
                        "avg_ms_without_first": sum(v[1:]) / max(1, len(v) - 1)} for k, v in dur.items()}
    json.dump({"source": f"prof_{tag}/trace", "launches_per_half": per_half, "launches": out["trace"],
               "note": "movie / user: per half-iteration, the sum of its main launches (one per slot chunk)"},
              open(os.path.join(dst, "main_launch_summary.json"), "w"), indent=1)
    # --- PMC passes ---
    def per_role(pattern):
        rows = load_rows(pattern)
        g = {int(r["Grid_Size"]) for r in rows if "als_solve_mfma" in r["Kernel_Name"] and not is_reduce(r["Kernel_Name"])
             and not is_fallback(r["Kernel_Name"])}
        hg = half_groups(rows, per_half)
        acc = defaultdict(lambda: defaultdict(list))
        disp = defaultdict(lambda: defaultdict(float))
        for r in rows:
            h = hg.get(int(r["Dispatch_Id"])) if hg else None
            if h:   # a half's chunk launches summed: counters per half-iteration, like the bench's launch time
                disp[(h[0], "half", h[1])][r["Counter_Name"]] += float(r["Counter_Value"])
                continue
            role = role_of(r["Kernel_Name"], int(r["Grid_Size"]), g)
            if role:
                disp[(role, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        for (role, *_), cnt in disp.items():
            for c, v in cnt.items():
                acc[role][c].append(v)
        return {role: {c: sum(v) / len(v) for c, v in cs.items()} for role, cs in acc.items()}
    fetch = per_role(f"{src}/fetch/**/*counter_collection.csv")
    write = per_role(f"{src}/write/**/*counter_collection.csv")
    traffic = {}
    for role in ("movie", "user", "reduce", "dual"):
        if role in fetch and role in write:
            traffic[role] = {"fetch_bytes_x2": fetch[role]["FETCH_SIZE"] * 1024 * 2,
                             "write_bytes": write[role]["WRITE_SIZE"] * 1024}
            traffic[role]["hbm_bytes"] = traffic[role]["fetch_bytes_x2"] + traffic[role]["write_bytes"]
    out["traffic"] = traffic
    for pas in ("sq", "sq_gram", "lds", "l2"):
        sq = per_role(f"{src}/{pas}/**/*counter_collection.csv")
        res = {}
        for role, c in sq.items():
            d = dict(c)
            if "SQ_LDS_BANK_CONFLICT" in c and "SQ_LDS_IDX_ACTIVE" in c and c["SQ_LDS_IDX_ACTIVE"] > 0:
                d["lds_bank_conflict_frac"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
            if "SQ_LDS_IDX_ACTIVE" in c and "GRBM_GUI_ACTIVE" in c:
                d["lds_active_frac"] = c["SQ_LDS_IDX_ACTIVE"] / (c["GRBM_GUI_ACTIVE"] / 8 * 256)   # per CU
            if "SQ_WAIT_INST_LDS" in c and "SQ_WAVE_CYCLES" in c:
                d["wait_inst_lds_frac"] = c["SQ_WAIT_INST_LDS"] / c["SQ_WAVE_CYCLES"]
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
                # MFMA busy cycles are summed over all SIMDs (1024); GRBM_GUI_ACTIVE over the 8 XCDs
                d["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024)
            if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c and c["TCC_HIT_sum"] + c["TCC_MISS_sum"] > 0:
                d["l2_hit_frac"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
            if "SQ_WAIT_INST_ANY" in c and "SQ_WAVE_CYCLES" in c:
                d["wait_inst_any_frac"] = c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"]
                d["wait_any_frac"] = c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"]
                d["active_inst_any_frac"] = c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
            res[role] = d
        out[pas] = res
    json.dump(out, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
    b = os.path.join(src, "bench.json")
    if os.path.exists(b):
        line = [l for l in open(b) if l.startswith("{")]
        if line:
            open(os.path.join(dst, "bench_line.json"), "w").write(line[-1])
    bench = json.loads(open(os.path.join(dst, "bench_line.json")).read()) if os.path.exists(os.path.join(dst, "bench_line.json")) else {}
    cfg = bench.get("config", {})
    k = cfg.get("k", 64)
    SIMDS, XCDS = 1024, 8
    per_side = {}
    for side in ("movie", "user"):
        sq, gr = out.get("sq", {}).get(side), out.get("sq_gram", {}).get(side)
        tr_ms = out["trace"].get(side, {}).get("avg_ms_without_first")
        d = {"hbm_bytes": traffic.get(side, {}).get("hbm_bytes"), "trace_avg_ms": tr_ms}
        if sq:
            cyc = sq["GRBM_GUI_ACTIVE"] / XCDS                   # GPU cycles of the launch (summed over XCDs)
            d["mfma_busy_frac"] = sq["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * SIMDS)
            d["valu_issue_frac"] = sq["SQ_INSTS_VALU"] / (cyc * SIMDS)
            d["mfma_mops"] = {x: sq[x] for x in ("SQ_INSTS_VALU_MFMA_MOPS_BF16", "SQ_INSTS_VALU_MFMA_MOPS_F16") if x in sq}
            d["wait_inst_any_frac"] = sq["SQ_WAIT_INST_ANY"] / sq["SQ_WAVE_CYCLES"]
            if tr_ms:
                d["clock_ghz"] = cyc / (tr_ms * 1e-3) / 1e9
            if gr:
                gcyc = gr["GRBM_GUI_ACTIVE"] / XCDS
                d["gram_only"] = {"cycles_frac": gcyc / cyc,
                                  "mfma_busy_frac": gr["SQ_VALU_MFMA_BUSY_CYCLES"] / (gcyc * SIMDS),
                                  "valu_issue_frac": gr["SQ_INSTS_VALU"] / (gcyc * SIMDS)}
                scyc = cyc - gcyc
                # the difference of two launches: meaningful only when the solve is a real share of the cycles (on the
                # gather-bound movie launch it is within the run-to-run noise of the Gram)
                if scyc > 0.05 * cyc:
                    d["solve_phase"] = {
                        "cycles_frac": scyc / cyc,
                        "mfma_busy_frac": (sq["SQ_VALU_MFMA_BUSY_CYCLES"] - gr["SQ_VALU_MFMA_BUSY_CYCLES"]) / (scyc * SIMDS),
                        "valu_issue_frac": (sq["SQ_INSTS_VALU"] - gr["SQ_INSTS_VALU"]) / (scyc * SIMDS),
                        "note": "whole launch minus the Gram-only launch of the same blocks (debug build)"}
        l2 = out.get("l2", {}).get(side)
        if l2 and "l2_hit_frac" in l2:
            d["l2_hit_frac"] = l2["l2_hit_frac"]
        ld = out.get("lds", {}).get(side)
        if ld:
            d["lds"] = {x: ld[x] for x in ("lds_bank_conflict_frac", "lds_active_frac", "wait_inst_lds_frac") if x in ld}
        per_side[side] = d
    json.dump({"k": k, "nnz": cfg.get("nnz", 100_000_000), "per_side": per_side, "source": f"profiles/{name}",
               "lib_sha256": bench.get("build", {}).get("lib_sha256"),
               "device_code_sha256": bench.get("build", {}).get("device_code_sha256"),
               "note": "per launch; hbm_bytes = FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, KiB -> B (Infinity-Cache "
                       "hits are counted by these counters); *_frac over 1024 SIMDs x the launch's GPU cycles "
                       "(GRBM_GUI_ACTIVE / 8 XCDs)"},
              open(os.path.join(ROOT, "profiles", counters_name(k, cfg)), "w"), indent=1)
    print(json.dumps({k: out[k] for k in ("trace", "traffic")}, indent=1))


if __name__ == "__main__":
    # optional: movie / user launches per half for a bench line that predates config.launches_per_half
    main(sys.argv[1], sys.argv[2],
         {"movie": int(sys.argv[3]), "user": int(sys.argv[4])} if len(sys.argv) > 4 else None)
