#!/bin/bash
# round 5 final tree: the whole GPU suite (every failure listed), then the
# p5 file alone
set -o pipefail
out=gpurun_out/r05zz
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/t.log 2>&1
rc=$?
tail -8 $out/t.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_p5.py -m gpu -v --timeout 300 --timeout-method thread > $out/p5.log 2>&1
tail -3 $out/p5.log
