#!/bin/bash
# A/B of the whole-tile pm_linear_jit variant (PM_JIT_WAVE=1): parity first
set -o pipefail
tag=${1:-wave}; out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
PM_JIT_WAVE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "specialized or multi_tile or pipelined" \
  --timeout 120 --timeout-method thread > "$out/t.log" 2>&1 || { tail -30 "$out/t.log"; exit 1; }
tail -2 "$out/t.log"
bash tools/gpu_ab.sh "$tag/ab" PM_JIT_WAVE=1 --steps 20 --warmup 5
