#!/bin/bash
# round 5: report chunks (PM_REP_CHUNK 16384 / 8192 / 4096 candidates of
# list capacity per chunk) on configs[4] and configs[2], alternating
set -o pipefail
out=gpurun_out/r05aj
mkdir -p $out
export TMPDIR=/tmp
for r in 1 2; do
for c in 16384 8192 4096; do
PM_REP_CHUNK=$c timeout -k 10 300 python3 bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline > $out/c4_${c}_$r.json 2> $out/c4_${c}_$r.err || { tail -20 $out/c4_${c}_$r.err; exit 1; }
PM_REP_CHUNK=$c timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/c2_${c}_$r.json 2> $out/c2_${c}_$r.err || { tail -20 $out/c2_${c}_$r.err; exit 1; }
echo "chunk $c run $r cfg4 $(python3 -c "import json;print(json.load(open('$out/c4_${c}_$r.json'))['ms_per_step'])") cfg2 $(python3 -c "import json;print(json.load(open('$out/c2_${c}_$r.json'))['ms_per_step'])")"
done
done
