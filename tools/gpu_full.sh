#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel stats, HBM
# traffic passes.  Usage: bash tools/gpu_full.sh <tag>
set -o pipefail
tag=${1:-run}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
echo "[tests]"
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
echo "[bench]"
timeout -k 10 300 python -u bench.py > "$out/bench.json" 2> "$out/bench.err" || { echo "bench failed"; tail -20 "$out/bench.err"; exit 1; }
cat "$out/bench.json"
echo "[rocprof stats]"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$out/bench_prof.json" 2> "$out/bench_prof.err" || { echo "rocprof failed"; tail -20 "$out/bench_prof.err"; exit 1; }
find "$out/prof" -name "*kernel_stats.csv" -exec head -4 {} \; | cut -c1-200
echo "[traffic]"
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$out/b$i" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$out/b$i.json" 2> "$out/b$i.err" || { echo "pmc $grp failed"; tail -5 "$out/b$i.err"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$out/c$i" -o run -- python3 tools/calib_fetch.py > "$out/c$i.log" 2> "$out/c$i.err" || { echo "calib $grp failed"; tail -5 "$out/c$i.err"; exit 1; }
done
echo done
