#!/bin/bash
# round 5: the ordered batch verify's retry and fallback paths
set -o pipefail
out=gpurun_out/r05ai
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_report.py -m gpu -x -v --timeout 300 --timeout-method thread -k "batch or config4 or ordered" > $out/t.log 2>&1 || { tail -40 $out/t.log; exit 1; }
tail -3 $out/t.log
