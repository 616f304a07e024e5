"""Round evidence (tools/gpu_evidence.sh output) -> committed files under
profiles/: bench lines, rocprofv3 kernel stats, PMC summaries of the two
hot kernels, the corrected HBM traffic of pm_linear_jit (FETCH_SIZE x 2 +
WRITE_SIZE, MI355X_MICROARCH.md HBM section, calibrated on known reads) and
the configs[0]/[1]/[3] timings.

usage: python tools/evidence_summary.py gpurun_out/<tag> <round>"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

root, rnd = sys.argv[1], sys.argv[2]
prof = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")


def copy(src, dst):
    if os.path.exists(src):
        shutil.copy(src, os.path.join(prof, dst))


def pmc(dirs, needle, grid=None):
    """Median counters per dispatch of the kernels named `needle` (of grid
    size `grid` when given: one bench run holds several workloads)."""
    agg, dur, grbm = {}, [], []
    for d in dirs:
        for f in glob.glob(os.path.join(root, d, "*counter_collection.csv")) + \
                glob.glob(os.path.join(root, d, "*", "*counter_collection.csv")):
            for row in csv.DictReader(open(f)):
                if needle not in row["Kernel_Name"] or (grid is not None and row["Grid_Size"] != grid):
                    continue
                agg.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
                dur.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    out = {k: statistics.median(v) for k, v in sorted(agg.items())}
    out["median_dispatch_ms"] = statistics.median(dur) * 1e3 if dur else None
    if "GRBM_GUI_ACTIVE" in out and dur:
        out["effective_clock_ghz"] = out["GRBM_GUI_ACTIVE"] / 8 / statistics.median(dur) / 1e9
    return out


def grids(d, needle):
    """Grid sizes of `needle`'s dispatches in order of first appearance."""
    seen = []
    for f in glob.glob(os.path.join(root, d, "*counter_collection.csv")) + \
            glob.glob(os.path.join(root, d, "*", "*counter_collection.csv")):
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
        for row in rows:
            if needle in row["Kernel_Name"] and row["Grid_Size"] not in seen:
                seen.append(row["Grid_Size"])
    return seen


for name in ("bench", "bench_ids", "configs"):
    copy(os.path.join(root, name + ".json"), "%s_%s.json" % (rnd, name))
for d in ("prof", "prof_ids"):
    copy(os.path.join(root, d, "run_kernel_stats.csv"), "%s_%s_kernel_stats.csv" % (rnd, d))
copy(os.path.join(root, "prof", "run_kernel_trace.csv"), "%s_prof_kernel_trace.csv" % rnd)
copy(os.path.join(root, "cfg3", "run_kernel_stats.csv"), "%s_cfg3_kernel_stats.csv" % rnd)
copy(os.path.join(root, "cfg3", "run_kernel_trace.csv"), "%s_cfg3_kernel_trace.csv" % rnd)
copy(os.path.join(root, "cfg3.log"), "%s_cfg3_query_ms.txt" % rnd)

lin = pmc(["p1", "p2"], "pm_linear_jit")
ids = pmc(["q1", "q2", "q3", "q4"], "pm_ids_rev")
batch = pmc(["c1", "c2"], "k_batch_scan")
# the same configs[4] passes hold every kernel of the step
cfg4 = {"%s (configs[4], 256 patterns k=0)" % k: pmc(["c1", "c2"], k)
        for k in ("k_batch_scan", "k_batch_verify_ord", "k_others_batch", "k_list_scatter", "k_rep_walk")}
cfg4["note"] = ("medians per dispatch from tools/gpu_evidence.sh's configs[4] passes (two counter groups); "
                "the exception pass runs beside the scan and verify on its own stream, so its and the verify's "
                "cycles include that overlap")
json.dump(cfg4, open(os.path.join(prof, "%s_cfg4_pmc.json" % rnd), "w"), indent=1)
cal = pmc(["cal"], "k_read")
bench = json.load(open(os.path.join(root, "bench.json")))
cal_bytes = json.load(open(os.path.join(root, "cal.json")))["bytes_per_launch"]
calib = {"bytes_read_per_launch": cal_bytes, "fetch_size_kb_median": cal.get("FETCH_SIZE"),
         "fetch_size_over_bytes": round(cal.get("FETCH_SIZE", 0) * 1024 / cal_bytes, 4)}
# FETCH_SIZE / WRITE_SIZE passes p3 / p4 ran the default bench (headline,
# then configs4, then the 100 Gbp extra): each workload's dominant kernel
# told apart by grid size, in that order
lg, bg = grids("p3", "pm_linear_jit"), grids("p3", "k_batch_scan")
work = [(bench, "pm_linear_jit", lg[0] if lg else None)]
if bench.get("configs4") and bg:
    work.append((bench["configs4"], "k_batch_scan", bg[0]))
if bench.get("north_star_100gbp") and len(lg) > 1:
    work.append((bench["north_star_100gbp"], "pm_linear_jit", lg[1]))
entries = []
for line, kern, grid in work:
    c = pmc(["p3", "p4"], kern, grid)
    alg = line["roofline"]["algorithmic_bytes_per_launch"]
    traffic = int(c["FETCH_SIZE"] * 1024 * 2 + c["WRITE_SIZE"] * 1024) if "FETCH_SIZE" in c and "WRITE_SIZE" in c else None
    wl = line["config"]["workload"] if "config" in line else line["workload"]
    entries.append({"workload": wl, "kernel": kern, "grid_size": int(grid) if grid else None,
                    "hbm_bytes_per_launch": traffic, "algorithmic_bytes_per_launch": alg,
                    "traffic_over_algorithmic": round(traffic / alg, 4) if traffic else None,
                    "fetch_size_kb_median": c.get("FETCH_SIZE"), "write_size_kb_median": c.get("WRITE_SIZE"),
                    "correction": "gfx950: FETCH_SIZE reports 1/2 of the bytes of 16 B/lane reads (global_load_dwordx4 "
                                  "and global_load_lds_dwordx4 alike, calibrated below); bytes = FETCH_SIZE*1024*2 + "
                                  "WRITE_SIZE*1024",
                    "calibration": calib,
                    "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes over the default bench "
                              "run (tools/gpu_evidence.sh p3 / p4)"})
idt = pmc(["q3", "q4"], "pm_ids_rev")
if "FETCH_SIZE" in idt and "WRITE_SIZE" in idt:
    bi = json.load(open(os.path.join(root, "bench_ids.json")))
    alg = bi["roofline"]["algorithmic_bytes_per_launch"]
    t = int(idt["FETCH_SIZE"] * 1024 * 2 + idt["WRITE_SIZE"] * 1024)
    entries.append({"workload": bi["config"]["workload"], "kernel": "pm_ids_rev", "hbm_bytes_per_launch": t,
                    "algorithmic_bytes_per_launch": alg, "traffic_over_algorithmic": round(t / alg, 4),
                    "fetch_size_kb_median": idt["FETCH_SIZE"], "write_size_kb_median": idt["WRITE_SIZE"],
                    "calibration": calib, "source": "rocprofv3 --pmc, passes q3 / q4"})
json.dump(entries, open(os.path.join(prof, "%s_traffic.json" % rnd), "w"), indent=1)
traffic = entries[0]["hbm_bytes_per_launch"] if entries else None
alg = entries[0]["algorithmic_bytes_per_launch"] if entries else None
json.dump({"pm_linear_jit (configs[2], k=2 substitutions)": lin, "pm_ids_rev (configs[2], -k 2ids)": ids,
           "k_batch_scan (configs[4], 256 patterns k=0)": batch,
           "note": "medians per dispatch; SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles "
                   "(MI355X_MICROARCH.md); one counter group per rocprofv3 run"},
          open(os.path.join(prof, "%s_pmc.json" % rnd), "w"), indent=1)
print(json.dumps({"traffic": traffic, "alg": alg, "lin_valu": lin.get("SQ_INSTS_VALU"),
                  "ids_valu": ids.get("SQ_INSTS_VALU"), "cal": cal.get("FETCH_SIZE")}))
# the steady-state dispatch means of the three workloads from the default
# run's kernel trace (tools/steady_state.py)
trace, line = os.path.join(root, "prof", "run_kernel_trace.csv"), os.path.join(root, "prof.json")
if os.path.exists(trace) and os.path.exists(line):
    import subprocess
    out = subprocess.run([sys.executable, os.path.join(os.path.dirname(os.path.abspath(__file__)), "steady_state.py"),
                          trace, line, "20"], capture_output=True, text=True, check=True).stdout
    open(os.path.join(prof, "%s_steady_state.json" % rnd), "w").write(out)
