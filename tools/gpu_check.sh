#!/bin/bash
# GPU-box routine: parity tests, bench, rocprofv3 kernel-trace summary.
# Usage (from the repo root on the box): bash tools/gpu_check.sh <tag> [bench args...]
set -o pipefail
tag=${1:-run}; shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -m gpu -x > "$out/gpu_tests.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
timeout -k 10 600 python bench.py "$@" > "$out/bench.json" 2> "$out/bench.err" || { echo "bench failed"; tail -20 "$out/bench.err"; exit 1; }
cat "$out/bench.json"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > "$out/bench_prof.json" 2> "$out/bench_prof.err" || { echo "rocprof failed"; tail -20 "$out/bench_prof.err"; exit 1; }
find "$out/prof" -name "*kernel_stats.csv" -exec head -8 {} \;
