#!/bin/bash
# configs[2] iteration + A/B of the DMA'd halo (full vs the words a window reads).
# usage: bash tools/gpu_halo.sh <tag>
set -o pipefail
bash tools/gpu_cfg2.sh "$1" || exit 1
for h in 1 0; do
  if [ $h = 1 ]; then export PM_JIT_FULL_HALO=1; else unset PM_JIT_FULL_HALO; fi
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/$1/b_h$h.json || exit 1
  echo "full_halo=$h $(grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"frac": [0-9.]*' gpurun_out/$1/b_h$h.json | tr '\n' ' ')"
done
