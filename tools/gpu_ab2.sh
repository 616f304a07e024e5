#!/bin/bash
# A/B/C/D of env knobs on the configs[2] bench (alternating runs on one box).
# Usage: bash tools/gpu_ab2.sh <tag> "<VAR=VAL ...>" ["<VAR=VAL ...>" ...]
set -o pipefail
out=gpurun_out/${1:-ab2}; shift
mkdir -p "$out"
export TMPDIR=/tmp
for i in 1 2; do
  j=0
  for knobs in "PM_NONE=0" "$@"; do
    j=$((j + 1))
    env $knobs timeout -k 10 120 python bench.py --no-cpu-baseline --steps 60 --warmup 5 > "$out/v${j}_$i.json" 2> "$out/v${j}_$i.err" || { echo "bench $knobs failed"; tail -5 "$out/v${j}_$i.err"; exit 1; }
    python - "$out/v${j}_$i.json" "$knobs" <<'PY'
import json, sys
a = json.load(open(sys.argv[1]))
print("%-28s %.4f ms/step kernel %.4f hits %s" % (sys.argv[2], a["ms_per_step"], a["roofline"]["kernel_ms"], a["config"].get("hits")))
PY
  done
done
