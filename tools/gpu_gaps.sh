#!/bin/bash
# configs[2] per-step gaps under env knobs: rocprofv3 kernel trace per variant
# Usage: bash tools/gpu_gaps.sh <tag> "<VAR=VAL ...>" ...
set -o pipefail
out=gpurun_out/${1:-gaps}; shift
mkdir -p "$out"
export TMPDIR=/tmp
j=0
for knobs in "PM_NONE=0" "$@"; do
  j=$((j + 1))
  env $knobs timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 --warmup 5 > "$out/b$j.json" 2> "$out/b$j.err" || { tail -5 "$out/b$j.err"; exit 1; }
  python3 -c "import json,sys; a=json.load(open(sys.argv[1])); print('%-34s %.4f ms/step kernel %.4f' % (sys.argv[2], a['ms_per_step'], a['roofline']['kernel_ms']))" "$out/b$j.json" "$knobs"
  env $knobs timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$out/t$j" -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > "$out/t$j.json" 2> "$out/t$j.err" || { tail -5 "$out/t$j.err"; exit 1; }
  python3 tools/step_gaps.py "$out/t$j/run_kernel_trace.csv"
  python3 tools/step_timeline.py "$out/t$j/run_kernel_trace.csv"
done
