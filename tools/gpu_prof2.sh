#!/bin/bash
# configs[2] bench + kernel stats (quick look at the step's kernels)
set -o pipefail
out=gpurun_out/${1:-prof2}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$out/bench.json" 2> "$out/bench.err" || { tail -5 "$out/bench.err"; exit 1; }
cut -c1-300 "$out/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > "$out/prof.json" 2> "$out/prof.err" || { tail -5 "$out/prof.err"; exit 1; }
python3 - "$out/prof/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print("%-60s n=%5s avg=%8.1f us tot=%8.2f ms" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
