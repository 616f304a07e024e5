#!/bin/bash
# round 5: the eregular engine (k > 0) on the GPU against the oracle
set -o pipefail
out=gpurun_out/r05d
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_regular.py -m gpu -v -x --timeout 300 --timeout-method thread > $out/t.log 2>&1
rc=$?
tail -40 $out/t.log
exit $rc
