#!/bin/bash
# round 5: the ordered batch verify (position-ordered lists, one stable
# pattern pass + merge instead of the whole-list radix sort) -- batch tests,
# configs[4] A/B, kernel stats
set -o pipefail
out=gpurun_out/r05w
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_report.py tests/test_gpu_parity.py tests/test_gpu_p5.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/t.log 2>&1 || { tail -40 $out/t.log; exit 1; }
tail -2 $out/t.log
timeout -k 10 300 python3 bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline > $out/bench4.json 2> $out/bench4.err || { tail -20 $out/bench4.err; exit 1; }
cut -c1-300 $out/bench4.json
PM_BATCH_EXC_CONC=1 timeout -k 10 300 python3 bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline > $out/bench4_off.json 2> $out/bench4_off.err || { tail -20 $out/bench4_off.err; exit 1; }
cut -c1-300 $out/bench4_off.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof4 -o run -- python3 bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline > $out/prof4.json 2> $out/prof4.err || { tail -20 $out/prof4.err; exit 1; }
python3 tools/kstats.py $out/prof4/run_kernel_stats.csv | head -30
