#!/bin/bash
# One GPU-box iteration: every -m gpu test (failures reported, a crash or
# timeout ends the call), then the default bench and its rocprofv3 kernel
# stats.  usage: bash tools/gpu_round.sh <tag> [extra bench args...]
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/$1; shift
mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $o/gpu_tests.txt 2>&1
rc=$?
tail -8 $o/gpu_tests.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py "$@" > $o/bench.json 2> $o/bench.err || { tail -20 $o/bench.err; exit 1; }
cut -c1-600 $o/bench.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > $o/bench_prof.json 2> $o/bench_prof.err || { tail -20 $o/bench_prof.err; exit 1; }
python3 tools/kstats.py $o/prof/run_kernel_stats.csv
