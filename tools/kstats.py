"""Print a rocprofv3 kernel_stats.csv as name / calls / mean us / total ms."""
import csv
import sys

for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    for r in rows[:24]:
        print("%-64s %5s %10.1f us %9.2f ms" % (r["Name"][:64], r["Calls"], float(r["AverageNs"]) / 1e3,
                                               float(r["TotalDurationNs"]) / 1e6))
