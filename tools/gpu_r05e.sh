#!/bin/bash
# round 5: pm_linear_jit with the parts rotating over the waves -- parity,
# then an alternating A/B against the fixed parts (PM_JIT_ROTATE=0), then a
# rocprof kernel trace of the default bench
set -o pipefail
out=gpurun_out/r05e
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_jit_shift.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -3 $out/t.log
bash tools/gpu_envab.sh r05e/ab PM_JIT_ROTATE=0 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
find $out/prof -name "*kernel_stats.csv" | head -3
