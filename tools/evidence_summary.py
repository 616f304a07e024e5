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


def pmc(dirs, needle):
    agg, dur, grbm = {}, [], []
    for d in dirs:
        for f in glob.glob(os.path.join(root, d, "*counter_collection.csv")) + \
                glob.glob(os.path.join(root, d, "*", "*counter_collection.csv")):
            for row in csv.DictReader(open(f)):
                if needle not in row["Kernel_Name"]:
                    continue
                agg.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
                dur.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    out = {k: statistics.median(v) for k, v in sorted(agg.items())}
    out["median_dispatch_ms"] = statistics.median(dur) * 1e3 if dur else None
    if "GRBM_GUI_ACTIVE" in out and dur:
        out["effective_clock_ghz"] = out["GRBM_GUI_ACTIVE"] / 8 / statistics.median(dur) / 1e9
    return out


for name in ("bench", "bench100", "bench_ids", "bench_cfg4", "configs"):
    copy(os.path.join(root, name + ".json"), "%s_%s.json" % (rnd, name))
for d in ("prof", "prof100", "prof_ids", "prof_cfg4"):
    copy(os.path.join(root, d, "run_kernel_stats.csv"), "%s_%s_kernel_stats.csv" % (rnd, d))
copy(os.path.join(root, "prof", "run_kernel_trace.csv"), "%s_prof_kernel_trace.csv" % rnd)
copy(os.path.join(root, "cfg3", "run_kernel_stats.csv"), "%s_cfg3_kernel_stats.csv" % rnd)
copy(os.path.join(root, "cfg3", "run_kernel_trace.csv"), "%s_cfg3_kernel_trace.csv" % rnd)
copy(os.path.join(root, "cfg3.log"), "%s_cfg3_query_ms.txt" % rnd)

lin = pmc(["p1", "p2", "p3", "p4"], "pm_linear_jit")
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
alg = bench["roofline"]["algorithmic_bytes_per_launch"]
cal_bytes = json.load(open(os.path.join(root, "cal.json")))["bytes_per_launch"]
traffic = None
if "FETCH_SIZE" in lin and "WRITE_SIZE" in lin:
    traffic = int(lin["FETCH_SIZE"] * 1024 * 2 + lin["WRITE_SIZE"] * 1024)
json.dump({"workload": bench["config"]["workload"], "kernel": "pm_linear_jit",
           "hbm_bytes_per_launch": traffic, "algorithmic_bytes_per_launch": alg,
           "traffic_over_algorithmic": round(traffic / alg, 4) if traffic else None,
           "fetch_size_kb_median": lin.get("FETCH_SIZE"), "write_size_kb_median": lin.get("WRITE_SIZE"),
           "correction": "gfx950: FETCH_SIZE reports 1/2 of the bytes of 16 B/lane reads (global_load_dwordx4 and "
                         "global_load_lds_dwordx4 alike, calibrated below); bytes = FETCH_SIZE*1024*2 + WRITE_SIZE*1024",
           "calibration": {"bytes_read_per_launch": cal_bytes, "fetch_size_kb_median": cal.get("FETCH_SIZE"),
                           "fetch_size_over_bytes": round(cal.get("FETCH_SIZE", 0) * 1024 / cal_bytes, 4)},
           "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes (tools/gpu_evidence.sh)"},
          open(os.path.join(prof, "%s_traffic.json" % rnd), "w"), indent=1)
json.dump({"pm_linear_jit (configs[2], k=2 substitutions)": lin, "pm_ids_rev (configs[2], -k 2ids)": ids,
           "k_batch_scan (configs[4], 256 patterns k=0)": batch,
           "note": "medians per dispatch; SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles "
                   "(MI355X_MICROARCH.md); one counter group per rocprofv3 run"},
          open(os.path.join(prof, "%s_pmc.json" % rnd), "w"), indent=1)
print(json.dumps({"traffic": traffic, "alg": alg, "lin_valu": lin.get("SQ_INSTS_VALU"),
                  "ids_valu": ids.get("SQ_INSTS_VALU"), "cal": cal.get("FETCH_SIZE")}))
