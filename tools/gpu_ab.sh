#!/bin/bash
# A/B of an env knob on the bench: alternating runs on one box.  Usage: bash tools/gpu_ab.sh <tag> <VAR=VAL> [bench args]
set -o pipefail
out=gpurun_out/${1:-ab}; knob=$2; shift 2
mkdir -p "$out"
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > "$out/a$i.json" 2> "$out/a$i.err" || { echo "bench A failed"; tail -5 "$out/a$i.err"; exit 1; }
  env $knob timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > "$out/b$i.json" 2> "$out/b$i.err" || { echo "bench B failed"; tail -5 "$out/b$i.err"; exit 1; }
  python - "$out/a$i.json" "$out/b$i.json" <<'PY'
import json, sys
a, b = (json.load(open(f)) for f in sys.argv[1:])
print("A %.4f ms/step kernel %.4f | B %.4f ms/step kernel %.4f" % (a["ms_per_step"], a["roofline"]["kernel_ms"], b["ms_per_step"], b["roofline"]["kernel_ms"]))
PY
done
