#!/bin/bash
# Experiment pass: report/parity tests (default and PM_OTHERS_BATCH=2), then
# kernel traces of configs[4] and of configs[2] with each exception-pass form.
# usage: bash tools/gpu_exp.sh <tag>
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/$1
mkdir -p $o
timeout -k 10 500 python -u -m pytest tests/test_gpu_report.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
PM_OTHERS_BATCH=2 timeout -k 10 500 python -u -m pytest tests/test_gpu_report.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $o/t2.log 2>&1 || { tail -30 $o/t2.log; exit 1; }
tail -1 $o/t2.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof4 -o run -- python3 bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline > $o/bench4.json 2> $o/prof4.err || exit 1
cut -c1-200 $o/bench4.json
for v in 1 2; do
  PM_OTHERS_BATCH=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof2_$v -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $o/bench2_$v.json 2> $o/prof2_$v.err || exit 1
  cut -c1-200 $o/bench2_$v.json
done
python3 - "$o" <<'PY'
import csv, sys
o = sys.argv[1]
for d in ("prof4", "prof2_1", "prof2_2"):
    print(d)
    for r in list(csv.DictReader(open(o + "/" + d + "/run_kernel_stats.csv")))[:10]:
        print("   %-50s %5s %8.3f" % (r["Name"][:50], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
