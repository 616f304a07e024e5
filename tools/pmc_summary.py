"""Summarise rocprofv3 --pmc CSVs for one kernel name substring."""
import collections
import csv
import glob
import sys

root, needle = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "k_linear")
agg = collections.defaultdict(list)
dur = []
for f in sorted(glob.glob(root + "/p*/run_counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        if needle not in row["Kernel_Name"]:
            continue
        agg[row["Counter_Name"]].append(float(row["Counter_Value"]))
        dur.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
for k, v in sorted(agg.items()):
    print("%-22s n=%-3d mean=%.4g" % (k, len(v), sum(v) / len(v)))
if dur:
    d = sorted(dur)[len(dur) // 2]
    print("median dispatch %.3f ms" % (d * 1e3))
    if "GRBM_GUI_ACTIVE" in agg:
        g = sorted(agg["GRBM_GUI_ACTIVE"])[len(agg["GRBM_GUI_ACTIVE"]) // 2]
        print("effective clock ~ %.2f GHz (GRBM_GUI_ACTIVE/8/dispatch)" % (g / 8 / d / 1e9))
