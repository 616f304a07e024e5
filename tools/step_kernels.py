"""Per-step kernel times of one workload from a rocprofv3 kernel trace:
the dispatches between consecutive launches of an anchor kernel (one per
step), summed per kernel name, the last `steps` steps; and one step's
timeline (start, end, queue, kernel).

usage: python tools/step_kernels.py <run_kernel_trace.csv> <anchor kernel substring> [steps] [grid]"""
import collections
import csv
import re
import sys


def name(n):
    n = n.replace("pm::(anonymous namespace)::", "").replace("void ", "")
    return re.split(r"[(<]", n)[0][:44]


def main():
    path, anchor = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    grid = sys.argv[4] if len(sys.argv) > 4 else None
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"] and (grid is None or r["Grid_Size_X"] == grid)]
    idx = idx[-(steps + 1):]
    tot, cnt = collections.Counter(), collections.Counter()
    for r in rows[idx[0]:idx[-1]]:
        nm = name(r["Kernel_Name"])
        tot[nm] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        cnt[nm] += 1
    n = len(idx) - 1
    span = (int(rows[idx[-1]]["Start_Timestamp"]) - int(rows[idx[0]]["Start_Timestamp"])) / 1e6
    print("steps %d, %.4f ms per step (anchor to anchor)" % (n, span / n))
    for k, v in tot.most_common(20):
        print("  %-44s %8.4f ms/step  %4.1f launches/step" % (k, v / n, cnt[k] / n))
    s0 = int(rows[idx[-2]]["Start_Timestamp"])
    print("one step:")
    for r in rows[idx[-2]:idx[-1]]:
        print("  %8.3f %8.3f q%s %s" % ((int(r["Start_Timestamp"]) - s0) / 1e6, (int(r["End_Timestamp"]) - s0) / 1e6,
                                        r["Queue_Id"], name(r["Kernel_Name"])))


if __name__ == "__main__":
    main()
