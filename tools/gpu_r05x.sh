#!/bin/bash
# round 5: configs[4] A/B -- the exception pass forked before the scan vs
# after it (beside the verify only), each run twice alternately
set -o pipefail
out=gpurun_out/r05x
mkdir -p $out
export TMPDIR=/tmp
for r in 1 2; do
for v in s v; do
PM_BATCH_EXC_AT=$v timeout -k 10 300 python3 bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline > $out/b_${v}_$r.json 2> $out/b_${v}_$r.err || { tail -20 $out/b_${v}_$r.err; exit 1; }
echo "$v $r $(python3 -c "import json;print(json.load(open('$out/b_${v}_$r.json'))['ms_per_step'])")"
done
done
