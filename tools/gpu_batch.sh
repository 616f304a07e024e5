#!/bin/bash
# Batch-path iteration: the batch parity tests, then a kernel trace of configs[4].
# usage: bash tools/gpu_batch.sh <tag>
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/$1
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_report.py -m gpu -x -q --timeout 300 --timeout-method thread -k batch > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof4 -o run -- python3 bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline > $o/bench4.json 2> $o/prof4.err || exit 1
cut -c1-200 $o/bench4.json
python3 - "$o" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1] + "/prof4/run_kernel_stats.csv")))[:10]:
    print("   %-50s %5s %8.3f" % (r["Name"][:50], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
