#!/bin/bash
# round 5 final tree: the whole GPU suite
set -o pipefail
out=gpurun_out/r05z
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/t.log 2>&1 || { tail -40 $out/t.log; exit 1; }
tail -3 $out/t.log
