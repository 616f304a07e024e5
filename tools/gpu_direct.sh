#!/bin/bash
# configs[2] iteration + A/B of the inline exception-bit selection.
# usage: bash tools/gpu_direct.sh <tag>
set -o pipefail
bash tools/gpu_cfg2.sh "$1" || exit 1
for d in 0 1; do
  PM_OTHERS_DIRECT=$d timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/$1/b_d$d.json || exit 1
  echo "direct=$d $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*' gpurun_out/$1/b_d$d.json | tr '\n' ' ')"
done
