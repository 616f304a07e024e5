#!/bin/bash
# round 5: huge bins radix-sorted by themselves (no whole-list radix sort),
# 16-position NFA chunks on small files -- the GPU suite, configs[4] bench +
# kernel trace, configs latency
set -o pipefail
out=gpurun_out/r05j
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/t.log 2>&1 || { tail -40 $out/t.log; exit 1; }
tail -2 $out/t.log
timeout -k 10 300 python3 bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline > $out/bench4.json 2> $out/bench4.err || { tail -20 $out/bench4.err; exit 1; }
cut -c1-400 $out/bench4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof4 -o run -- python3 bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline > $out/prof4.json 2> $out/prof4.err || { tail -20 $out/prof4.err; exit 1; }
python3 tools/kstats.py $out/prof4/run_kernel_stats.csv 2>/dev/null | head -20 || true
timeout -k 10 300 python3 tools/config_times.py > $out/configs.json 2> $out/configs.err || { tail -20 $out/configs.err; exit 1; }
cat $out/configs.json
