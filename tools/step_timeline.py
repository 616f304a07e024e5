"""One configs[2] step from a rocprofv3 kernel trace: every dispatch from
one pm_linear_jit start to the next, with its queue, start offset, duration
and the gap before it (microseconds)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
jit = [i for i, r in enumerate(rows) if r["Kernel_Name"] == "pm_linear_jit"]
a, b = jit[-3], jit[-2]
t0 = int(rows[a]["Start_Timestamp"])
prev_end = None
for r in rows[a:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    print("%8.1f %7.1f gap %6.1f q%-3s %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, r.get("Queue_Id", "?"),
                                             r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-40:]))
    prev_end = max(prev_end or 0, e)
