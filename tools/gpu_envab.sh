#!/bin/bash
# A/B of one env knob on the configs[2] bench (alternating, same library).
# Usage: bash tools/gpu_envab.sh <tag> VAR=VAL
set -o pipefail
out=gpurun_out/${1:-envab}; knob=$2
mkdir -p "$out"
for i in 1 2 3; do
  for v in base knob; do
    if [ $v = knob ]; then envs="$knob"; else envs="PM_NONE=0"; fi
    env $envs timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 --warmup 5 > "$out/$v$i.json" 2> "$out/$v$i.err" || { tail -5 "$out/$v$i.err"; exit 1; }
    python3 -c "import json,sys; a=json.load(open(sys.argv[1])); print('%-5s %.4f ms/step kernel %.4f frac %.4f hits %s' % (sys.argv[2], a['ms_per_step'], a['roofline']['kernel_ms'], a['roofline']['frac'], a['config'].get('hits')))" "$out/$v$i.json" $v
  done
done
