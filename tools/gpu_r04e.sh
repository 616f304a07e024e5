#!/bin/bash
# eextended (k > 0 extended patterns) on the GPU: its parity tests, then the
# whole -m gpu suite.
set -o pipefail
tag=${1:-r04e}; out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_eextended.py -m gpu -x -v --timeout 300 --timeout-method thread > "$out/ee.txt" 2>&1
rc=$?; tail -30 "$out/ee.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > "$out/all.txt" 2>&1
rc=$?; tail -8 "$out/all.txt"; exit $rc
