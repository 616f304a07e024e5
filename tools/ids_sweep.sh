#!/bin/bash
# A/B of the bit-sliced -k ids start pass' knobs (lane width, prefetch depth)
# usage: bash tools/ids_sweep.sh <tag> [lw list] [u list]
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
for lw in ${2:-64 32}; do
  for u in ${3:-2 4}; do
    PM_IDS_LW=$lw PM_IDS_U=$u timeout -k 10 200 python bench.py --types ids --steps 4 --warmup 1 --no-cpu-baseline > $out/lw${lw}_u${u}.json 2>/dev/null || { echo "lw=$lw u=$u failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$out/lw${lw}_u${u}.json'));print('lw=$lw u=$u', d['ms_per_step'], d['roofline']['kernel_ms'], d['config']['hits'])"
  done
done
