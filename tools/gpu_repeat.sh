#!/bin/bash
# Run-to-run spread of the default bench line (configs[2]) on one box:
# bench.py with no flags, 5 times back to back.
# usage: bash tools/gpu_repeat.sh <tag>
set -o pipefail
o=gpurun_out/$1
mkdir -p $o
for i in 1 2 3 4 5; do
  timeout -k 10 240 python bench.py > $o/bench_$i.json 2> $o/bench_$i.err || { tail -20 $o/bench_$i.err; exit 1; }
  tail -1 $o/bench_$i.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print($i, d['value'], d['ms_per_step'], r['achieved'], r['frac'])"
done
