#!/bin/bash
# round 5: the report walk's lane-flag header checks issued with the keys'
# loads -- the GPU suite, configs[4] bench + trace
set -o pipefail
out=gpurun_out/r05v
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/t.log 2>&1 || { tail -40 $out/t.log; exit 1; }
tail -2 $out/t.log
timeout -k 10 300 python3 bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline > $out/bench4.json 2> $out/bench4.err || { tail -20 $out/bench4.err; exit 1; }
cut -c1-300 $out/bench4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof4 -o run -- python3 bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline > $out/prof4.json 2> $out/prof4.err || { tail -20 $out/prof4.err; exit 1; }
python3 tools/kstats.py $out/prof4/run_kernel_stats.csv | grep -E "rep_|batch"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/bench2.json 2> $out/bench2.err || { tail -20 $out/bench2.err; exit 1; }
cut -c1-300 $out/bench2.json
