#!/bin/bash
# round 5, first call: the new oracle checks of the graded tail and the
# long shifted pair, then the default bench line (parity sample: both ends)
set -o pipefail
out=gpurun_out/r05a
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_graded.py tests/test_gpu_jit_shift.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/t.log 2>&1 || { tail -40 $out/t.log; exit 1; }
tail -15 $out/t.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
