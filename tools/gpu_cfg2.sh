#!/bin/bash
# configs[2] iteration: linear/report parity tests, then a kernel trace of the default bench.
# usage: bash tools/gpu_cfg2.sh <tag>
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/$1
mkdir -p $o
timeout -k 10 500 python -u -m pytest tests/test_gpu_report.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof2 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $o/bench2.json 2> $o/prof2.err || exit 1
cut -c1-200 $o/bench2.json
python3 - "$o" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1] + "/prof2/run_kernel_stats.csv")))[:8]:
    print("   %-50s %5s %8.3f" % (r["Name"][:50], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
