"""Per-step GPU timeline from a rocprofv3 kernel trace: kernel time of
pm_linear_jit vs everything between consecutive pm_linear_jit starts."""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
jit = [r for r in rows if r["Kernel_Name"] == "pm_linear_jit"]
periods, kern = [], []
for a, b in zip(jit, jit[1:]):
    periods.append((int(b["Start_Timestamp"]) - int(a["Start_Timestamp"])) / 1e3)
    kern.append((int(a["End_Timestamp"]) - int(a["Start_Timestamp"])) / 1e3)
periods, kern = periods[-8:], kern[-8:]
print("period us  median %.1f  kernel us median %.1f  other %.1f" % (
    statistics.median(periods), statistics.median(kern), statistics.median(p - k for p, k in zip(periods, kern))))
