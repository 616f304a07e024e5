#!/bin/bash
# Round-end evidence: GPU parity tests, the default bench line, the rocprofv3
# kernel-trace summary of the same command, idle-clock kernel timings.
# Usage: bash tools/gpu_final.sh <tag>
set -o pipefail
out=gpurun_out/${1:-final}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { echo "gpu tests failed"; tail -40 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
timeout -k 10 300 python bench.py > "$out/bench.json" 2> "$out/bench.err" || { echo "bench failed"; tail -20 "$out/bench.err"; exit 1; }
cat "$out/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- python3 bench.py > "$out/bench_prof.json" 2> "$out/bench_prof.err" || { echo "rocprof failed"; tail -20 "$out/bench_prof.err"; exit 1; }
cat "$out/bench_prof.json"
find "$out/prof" -name "*kernel_stats.csv" -exec cut -c1-120 {} \; | head -4
PM_SWEEP_GAP_MS=50 timeout -k 10 300 python -u tools/jit_sweep.py 10 TGCTGASTCAGCANW 2 "" "PM_JIT_NOSHARE=1" > "$out/idle_sweep.txt" 2>&1 || { echo "sweep failed"; tail -20 "$out/idle_sweep.txt"; exit 1; }
cat "$out/idle_sweep.txt"
