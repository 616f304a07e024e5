#!/bin/bash
# configs[4] A/B: fused scan+verify vs the separate verify pass, then batch tests
set -o pipefail
out=gpurun_out/${1:-cfg4ab}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_report.py -k "config4 or batch" > "$out/tests.txt" 2>&1 || { tail -30 "$out/tests.txt"; exit 1; }
tail -2 "$out/tests.txt"
for i in 1 2; do
  for f in 1 0; do
    PM_BATCH_FUSED=$f timeout -k 10 300 python bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline > "$out/b${f}_$i.json" 2> "$out/b${f}_$i.err" || { tail -5 "$out/b${f}_$i.err"; exit 1; }
    python - "$out/b${f}_$i.json" "$f" <<'PY'
import json, sys
a = json.load(open(sys.argv[1]))
print("fused=%s %.3f ms/step kernel %.3f hits %s" % (sys.argv[2], a["ms_per_step"], a["roofline"]["kernel_ms"], a["config"].get("hits")))
PY
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- python3 bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline > "$out/prof.json" 2> "$out/prof.err" || { tail -5 "$out/prof.err"; exit 1; }
python3 - "$out/prof/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print("%-60s n=%5s avg=%9.1f us tot=%8.2f ms" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
