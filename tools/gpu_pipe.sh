#!/bin/bash
# Pipelined-scan check: parity tests, bench pipelined vs serial, rocprof of the bench.
set -o pipefail
out=gpurun_out/${1:-pipe}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { echo "gpu tests failed"; tail -40 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
timeout -k 10 300 python bench.py > "$out/bench.json" 2> "$out/bench.err" || { echo "bench failed"; tail -20 "$out/bench.err"; exit 1; }
cat "$out/bench.json"
timeout -k 10 300 python bench.py --serial --no-cpu-baseline > "$out/bench_serial.json" 2> "$out/bench_serial.err" || { echo "bench serial failed"; tail -20 "$out/bench_serial.err"; exit 1; }
cat "$out/bench_serial.json"
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > "$out/bench50.json" 2> "$out/bench50.err" || { echo "bench50 failed"; tail -20 "$out/bench50.err"; exit 1; }
cat "$out/bench50.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$out/bench_prof.json" 2> "$out/bench_prof.err" || { echo "rocprof failed"; tail -20 "$out/bench_prof.err"; exit 1; }
find "$out/prof" -name "*kernel_stats.csv" -exec cut -c1-160 {} \; | head -6
