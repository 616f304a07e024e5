#!/bin/bash
# the tests that read e2e.json / the >64-position kernels, then the whole -m gpu suite
set -o pipefail
tag=${1:-r04s}; out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_service_gpu.py tests/test_gpu_wide.py -m gpu -x -q --timeout 300 --timeout-method thread > "$out/sw.txt" 2>&1
rc=$?; tail -30 "$out/sw.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > "$out/all.txt" 2>&1
rc=$?; tail -8 "$out/all.txt"; exit $rc
