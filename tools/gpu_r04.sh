#!/bin/bash
# round-4 GPU check: the new extended-engine tests, the whole -m gpu suite,
# then the pm_linear_jit waves-per-workgroup A/B (parity first).
set -o pipefail
tag=${1:-r04}; out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_extended.py -m gpu -x -v --timeout 240 --timeout-method thread > "$out/ext.txt" 2>&1
rc=$?; tail -4 "$out/ext.txt"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > "$out/all.txt" 2>&1
rc=$?; tail -6 "$out/all.txt"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_parts.sh "$tag/parts"
