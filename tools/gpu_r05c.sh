#!/bin/bash
# round 5: key-level multi-rank rehearsal (configs[2], -k 2ids, configs[4])
# and the regular engine
set -o pipefail
out=gpurun_out/r05c
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_ranks.py tests/test_gpu_regular.py -m gpu -v --timeout 400 --timeout-method thread > $out/t.log 2>&1
rc=$?
tail -25 $out/t.log
exit $rc
