"""One step's kernel timeline from a rocprofv3 kernel trace (the last full
step between two dispatches of the named kernel): start, duration, the GPU
idle gap before each kernel, queue."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
first = sys.argv[2] if len(sys.argv) > 2 else "k_batch_scan"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
i0, i1 = idx[-2], idx[-1]
t0 = int(rows[i0]["Start_Timestamp"])
end = t0
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = re.sub(r"\(.*", "", r["Kernel_Name"])
    name = re.sub(r"<.*", "", name.replace("void ", ""))[-40:]
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:8.1f} gap {max(0, s - end) / 1e3:7.1f} q{r['Queue_Id']} {name}")
    end = max(end, e)
print("step", (int(rows[i1]["Start_Timestamp"]) - t0) / 1e3, "us")
