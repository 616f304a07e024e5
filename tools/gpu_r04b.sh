#!/bin/bash
# the 2-rank bench rehearsal (one card shared by both ranks)
set -o pipefail
tag=${1:-r04b}; out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_ranks.py -m gpu -x -v --timeout 500 --timeout-method thread > "$out/ranks.txt" 2>&1
rc=$?; tail -25 "$out/ranks.txt"; exit $rc
