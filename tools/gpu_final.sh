#!/bin/bash
# Round-end check on one box: every GPU test, smoke(), then the evidence run.
# usage: bash tools/gpu_final.sh <tag>
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/$1
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.txt 2>&1 || { tail -30 $o/gpu_tests.txt; exit 1; }
tail -1 $o/gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.txt 2>&1 || { cat $o/smoke.txt; exit 1; }
cat $o/smoke.txt
bash tools/gpu_evidence.sh "$1"
