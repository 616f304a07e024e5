#!/bin/bash
# configs[4]: output segment size A/B (PM_BATCH_WPO scan waves per segment).
# usage: bash tools/gpu_wpo.sh <tag>
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/$1
mkdir -p $o
for w in ${WPOS:-1 2 4 8}; do
  PM_BATCH_WPO=$w timeout -k 10 200 python bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline > $o/b_w$w.json || exit 1
  echo "wpo=$w $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $o/b_w$w.json | tr '\n' ' ')"
done
PM_BATCH_WPO=${TWPO:-1} timeout -k 10 300 python -u -m pytest tests/test_gpu_report.py -m gpu -x -q --timeout 300 --timeout-method thread -k batch > $o/t1.log 2>&1 || { tail -20 $o/t1.log; exit 1; }
tail -1 $o/t1.log
