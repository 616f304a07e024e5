#!/bin/bash
# quick GPU iteration: parity/report tests, bench, kernel-trace profile
# usage: bash tools/gpu_quick.sh <tag> [pytest selection...]
set -o pipefail
tag=$1; shift
sel=${*:-tests/test_gpu_parity.py tests/test_gpu_report.py}
export TMPDIR=/tmp
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 400 python -u -m pytest $sel -m gpu -x -q --timeout 120 --timeout-method thread > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -2 $out/t.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/bench_prof.json 2> $out/bench_prof.err || exit 1
cut -c1-110 $out/prof/run_kernel_stats.csv | head -12
