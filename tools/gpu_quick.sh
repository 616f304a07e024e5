#!/bin/bash
# GPU-box quick loop: parity tests, then the specialized kernel timed on the
# bench workload under generator variants.  Usage: bash tools/gpu_quick.sh <tag> [variants...]
set -o pipefail
tag=${1:-quick}; shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { echo "gpu tests failed"; tail -40 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
timeout -k 10 300 python -u tools/jit_sweep.py 10 TGCTGASTCAGCANW 2 "$@" > "$out/sweep.txt" 2>&1 || { echo "sweep failed"; tail -20 "$out/sweep.txt"; exit 1; }
cat "$out/sweep.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- python3 tools/jit_sweep.py 10 TGCTGASTCAGCANW 2 "" > "$out/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$out/prof.log"; exit 1; }
find "$out/prof" -name "*kernel_stats.csv" -exec cut -c1-150 {} \; | head -12
