#!/bin/bash
# pm_linear_jit waves-per-workgroup A/B: parity of the 2-wave form, then
# alternating benches (A = default, B = PM_JIT_PARTS=2) and a kernel trace.
set -o pipefail
tag=${1:-parts}; out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
PM_JIT_PARTS=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "specialized or multi_tile or pipelined or sort_regimes" \
  --timeout 120 --timeout-method thread > "$out/t2.log" 2>&1 || { tail -30 "$out/t2.log"; exit 1; }
tail -2 "$out/t2.log"
bash tools/gpu_ab.sh "$tag/ab" PM_JIT_PARTS=2 --steps 20 --warmup 5 || exit 1
PM_JIT_PARTS=2 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof2" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$out/bench_prof2.json" 2> "$out/bench_prof2.err" || exit 1
cut -c1-110 "$out/prof2/run_kernel_stats.csv" | head -6
