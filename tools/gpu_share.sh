#!/bin/bash
# Shared-block experiment: parity, then the kernel with/without sharing
# (back to back and at the recovered clock), then the bench + rocprof.
set -o pipefail
out=gpurun_out/${1:-share}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { echo "gpu tests failed"; tail -40 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
timeout -k 10 300 python -u tools/jit_sweep.py 10 TGCTGASTCAGCANW 2 "" "PM_JIT_NOSHARE=1" "" "PM_JIT_NOSHARE=1" > "$out/sweep.txt" 2>&1 || { echo "sweep failed"; tail -20 "$out/sweep.txt"; exit 1; }
PM_SWEEP_GAP_MS=50 timeout -k 10 300 python -u tools/jit_sweep.py 10 TGCTGASTCAGCANW 2 "" "PM_JIT_NOSHARE=1" >> "$out/sweep.txt" 2>&1 || { echo "sweep gap failed"; tail -20 "$out/sweep.txt"; exit 1; }
cat "$out/sweep.txt"
timeout -k 10 300 python bench.py > "$out/bench.json" 2> "$out/bench.err" || { echo "bench failed"; tail -20 "$out/bench.err"; exit 1; }
cat "$out/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$out/bench_prof.json" 2> "$out/bench_prof.err" || { echo "rocprof failed"; tail -20 "$out/bench_prof.err"; exit 1; }
find "$out/prof" -name "*kernel_stats.csv" -exec cut -c1-160 {} \; | head -6
