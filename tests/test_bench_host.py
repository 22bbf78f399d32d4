"""bench.py's host-side contract pieces that need no GPU: counters are used only for the library they were profiled
with, the CPU-baseline legs never exceed the process's CPU share (item 7), and the diagnostics
build is refused before anything is measured."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _write_counters(tmp_path, monkeypatch, **fields):
    prof = tmp_path / "profiles"
    prof.mkdir()
    c = {"k": 64, "nnz": 1000, "lib_sha256": "a" * 64, "source": "profiles/rXX", "per_side": {}}
    c.update(fields)
    (prof / "counters_k64.json").write_text(json.dumps(c))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))


def test_counters_used_for_the_profiled_library_only(tmp_path, monkeypatch):
    _write_counters(tmp_path, monkeypatch)
    c, why = bench.load_counters(64, 1000, "a" * 64)
    assert c is not None and why is None
    c, why = bench.load_counters(64, 1000, "b" * 64)
    assert c is None and why.startswith("stale:") and "aaaaaaaaaaaa" in why and "bbbbbbbbbbbb" in why


def test_counters_follow_the_device_code_across_host_only_rebuilds(tmp_path, monkeypatch):
    """counters stamped with the profiled library's device-code hash stay valid for a library whose host code
    changed but whose .hip_fatbin (the kernels) did not; a different device code drops them"""
    _write_counters(tmp_path, monkeypatch, device_code_sha256="d" * 64)
    c, why = bench.load_counters(64, 1000, "b" * 64, dev_sha="d" * 64)
    assert c is not None and why is None and c["matched_by"] == "device_code_sha256"
    c, why = bench.load_counters(64, 1000, "b" * 64, dev_sha="e" * 64)
    assert c is None and why.startswith("stale:")


def test_device_code_hash_reads_the_fatbin_section(cfk):
    """__graft_entry__.device_code_sha256 = sha256 of the library's .hip_fatbin section, as llvm-objcopy dumps it"""
    import subprocess
    import hashlib
    import __graft_entry__
    from cfk_amd import _lib
    path = os.path.realpath(_lib.LIB_PATH)
    out = os.path.join(os.path.dirname(path), "fatbin_test.bin")
    try:
        subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objcopy", "--dump-section", f".hip_fatbin={out}", path,
                        out + ".so"], check=True)
        assert __graft_entry__.device_code_sha256(path) == hashlib.sha256(open(out, "rb").read()).hexdigest()
    finally:
        for f in (out, out + ".so"):
            if os.path.exists(f):
                os.remove(f)


def test_counters_of_another_workload_are_dropped(tmp_path, monkeypatch):
    _write_counters(tmp_path, monkeypatch)
    assert bench.load_counters(64, 2000, "a" * 64)[0] is None
    (tmp_path / "profiles" / "counters_k64.json").unlink()
    c, why = bench.load_counters(64, 1000, "a" * 64)
    assert c is None and why.startswith("no ")


def test_committed_counters_carry_a_library_hash():
    for k in (64, 128):
        c = json.load(open(os.path.join(ROOT, "profiles", f"counters_k{k}.json")))
        assert c["k"] == k and len(c["lib_sha256"]) == 64, k
        assert set(c["per_side"]) >= {"movie", "user"}, k


def test_cpu_share_honours_affinity_and_omp(monkeypatch):
    monkeypatch.delenv("OMP_NUM_THREADS", raising=False)
    n, src = bench.cpu_share()
    assert 1 <= n <= len(os.sched_getaffinity(0)) and src.startswith("affinity")
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    n3, src3 = bench.cpu_share()
    assert n3 == min(3, n) and "OMP_NUM_THREADS 3" in src3


@pytest.mark.parametrize("copy", [False, True])
def test_bench_refuses_the_debug_library(tmp_path, copy):
    """Refused by what the library exports (als_debug_knobs_compiled, debug build only), not by its path: a copy of
    the diagnostics build under another name is refused too."""
    import shutil
    lib = os.path.join(ROOT, "collaborative-filtering-kafka_amd", "build_debug", "libcfk_als.so")
    if copy:
        shutil.copy(lib, tmp_path / "libcfk_als.so")
        lib = str(tmp_path / "libcfk_als.so")
    env = dict(os.environ, CFK_ALS_LIB=lib)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "refused" in r.stderr, r.stderr[-2000:]


def test_prof_summary_sums_the_chunk_launches_of_each_half(tmp_path, monkeypatch):
    """tools/prof_summary.py on a chunked run (bench config launches_per_half = 2 movie + 3 user launches per
    iteration): the trace summary and the per-half counters are sums over each half-iteration's launches, in dispatch
    order, and the counters file is stamped with the profiled library's hashes"""
    import csv
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import prof_summary
    monkeypatch.setattr(prof_summary, "ROOT", str(tmp_path))
    src = tmp_path / "gpurun_out" / "prof_t"
    main_k = "void cfk::(anonymous namespace)::als_solve_mfma<64, 2, true, false, false, false>(x)"
    red_k = "void cfk::(anonymous namespace)::als_solve_mfma<64, 2, false, false, true, false>(x)"
    rows, pmc, did, t = [], [], 0, 0
    for it in range(3):
        for half, n in (("movie", 2), ("user", 3)):
            for c in range(n):
                did += 1
                dur = 1_000_000 if half == "movie" else 2_000_000   # ns: movie half 2 ms, user half 6 ms
                rows.append({"Kernel_Name": main_k, "Dispatch_Id": did, "Grid_Size_X": 100 + c,
                             "Start_Timestamp": t, "End_Timestamp": t + dur})
                for cnt, v in (("FETCH_SIZE", 10.0), ("WRITE_SIZE", 1.0)):
                    pmc.append({"Kernel_Name": main_k, "Dispatch_Id": did, "Grid_Size": 100 + c,
                                "Counter_Name": cnt, "Counter_Value": v})
                t += dur
                did += 1
                rows.append({"Kernel_Name": red_k, "Dispatch_Id": did, "Grid_Size_X": 7,
                             "Start_Timestamp": t, "End_Timestamp": t + 1000})
    for sub, data, fields in (("trace/run_kernel_trace.csv", rows, rows[0].keys()),
                              ("fetch/run_counter_collection.csv", [r for r in pmc if r["Counter_Name"] == "FETCH_SIZE"], pmc[0].keys()),
                              ("write/run_counter_collection.csv", [r for r in pmc if r["Counter_Name"] == "WRITE_SIZE"], pmc[0].keys())):
        p = src / sub
        p.parent.mkdir(parents=True, exist_ok=True)
        with open(p, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(fields))
            w.writeheader()
            w.writerows(data)
    line = {"config": {"k": 64, "nnz": 1000, "workload_name": "netflix", "launches_per_half": {"movie": 2, "user": 3}},
            "build": {"lib_sha256": "a" * 64, "device_code_sha256": "d" * 64}}
    (src / "bench.json").write_text(json.dumps(line) + "\n")
    prof_summary.main("t", "rT")
    tr = json.load(open(tmp_path / "profiles" / "rT" / "main_launch_summary.json"))["launches"]
    assert tr["movie"]["calls"] == 3 and abs(tr["movie"]["avg_ms"] - 2.0) < 1e-9
    assert tr["user"]["calls"] == 3 and abs(tr["user"]["avg_ms"] - 6.0) < 1e-9
    c = json.load(open(tmp_path / "profiles" / "counters_k64.json"))
    assert c["per_side"]["movie"]["hbm_bytes"] == 2 * (10 * 1024 * 2 + 1024)
    assert c["per_side"]["user"]["hbm_bytes"] == 3 * (10 * 1024 * 2 + 1024)
    assert c["lib_sha256"] == "a" * 64 and c["device_code_sha256"] == "d" * 64


def test_roofline_source_labels():
    """Where a half's gathered rows come from and the label its roofline line carries: the
    configs[4] user table (2.56 GB, beyond the 256 MiB Infinity Cache) is a mixed IC/HBM figure, not a pure HBM
    bound; an interleaved half walks its IC-resident table in step (priced against the L2 ceiling)."""
    assert bench.served_from(17_771 * 256, False) == ("l2", bench.L2_GATHER_CEILING_GBS)
    assert bench.served_from(480_190 * 256, False) == ("ic", bench.IC_GATHER_CEILING_GBS)
    assert bench.served_from(10_000_001 * 256, False) == ("hbm", bench.HBM_PEAK_GBS)
    assert bench.served_from(480_190 * 256, True) == ("l2_ic_walk", bench.L2_GATHER_CEILING_GBS)
    assert bench.bound_label("hbm") == "beyond_ic_mixed"
    assert bench.bound_label("l2_ic_walk") == "l2_ic_walk_gather"
    assert bench.bound_label("ic") == "ic_gather"
    assert bench.HBM_MEASURED_GBS < bench.HBM_PEAK_GBS
