#!/bin/bash
# -k ids iteration: bit-sliced start-pass parity tests, bench line, kernel trace
# usage: bash tools/gpu_ids.sh <tag>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ids.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -1 $out/t.log
timeout -k 10 300 python bench.py --types ids --steps 5 --warmup 2 --no-cpu-baseline > $out/bench_ids.json 2> $out/bench_ids.err || { tail -20 $out/bench_ids.err; exit 1; }
cut -c1-400 $out/bench_ids.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py --types ids --steps 5 --warmup 2 --no-cpu-baseline > $out/bench_ids_prof.json 2>&1 || exit 1
cut -c1-110 $out/prof/run_kernel_stats.csv | head -5
