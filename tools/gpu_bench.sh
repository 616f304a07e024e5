#!/bin/bash
# Bench recipe: selected GPU tests, then the default bench, the -k 2ids
# bench and a kernel-trace profile of the default bench.  Any step that
# times out or crashes ends the call (pytest failures go on).
# usage: tools/gpu_bench.sh <tag> [pytest targets...]
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
if [ $# -gt 0 ]; then
    timeout -k 10 700 python -u -m pytest "$@" -q -rf --timeout 240 --timeout-method thread > "$out/tests.txt" 2>&1
    rc=$?; echo "tests rc=$rc" >> "$out/status.txt"; tail -3 "$out/tests.txt"
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
timeout -k 10 300 python -u bench.py > "$out/bench.json" 2> "$out/bench.err"
rc=$?; echo "bench rc=$rc" >> "$out/status.txt"; cat "$out/bench.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --types ids > "$out/bench_ids.json" 2> "$out/bench_ids.err"
rc=$?; echo "bench_ids rc=$rc" >> "$out/status.txt"; cat "$out/bench_ids.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- python3 bench.py --steps 20 --no-cpu-baseline > "$out/prof_bench.json" 2> "$out/prof.err"
rc=$?; echo "prof rc=$rc" >> "$out/status.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_ids" -o run -- python3 bench.py --types ids --steps 10 --no-cpu-baseline > "$out/prof_ids_bench.json" 2> "$out/prof_ids.err"
rc=$?; echo "prof_ids rc=$rc" >> "$out/status.txt"
find "$out" -name "*kernel_stats.csv" | head
