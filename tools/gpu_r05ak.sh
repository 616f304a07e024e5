#!/bin/bash
# round 5 final tree: back-to-back default bench runs (configs[2]) and
# configs[4] runs on one box -- the run-to-run spread
set -o pipefail
out=gpurun_out/r05ak
mkdir -p $out
export TMPDIR=/tmp
for r in 1 2 3 4; do
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $out/c2_$r.json 2> $out/c2_$r.err || { tail -20 $out/c2_$r.err; exit 1; }
timeout -k 10 300 python3 bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline > $out/c4_$r.json 2> $out/c4_$r.err || { tail -20 $out/c4_$r.err; exit 1; }
python3 - "$out" "$r" <<'PY'
import json, sys
o, r = sys.argv[1], sys.argv[2]
a = json.load(open("%s/c2_%s.json" % (o, r))); b = json.load(open("%s/c4_%s.json" % (o, r)))
print("run %s configs[2] %.1f Gbases/s %.4f ms (frac %.3f) | configs[4] %.1f Gbases/s %.4f ms" % (
    r, a["value"], a["ms_per_step"], a["roofline"]["frac"], b["value"], b["ms_per_step"]))
PY
done
