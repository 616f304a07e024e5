#!/bin/bash
# Quick GPU iteration: the given pytest files, then bench lines with their
# rocprofv3 kernel stats.  usage: bash tools/gpu_iter.sh <tag> "<pytest files>" "<bench args>" ["<bench args>" ...]
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/$1; tests=$2; shift 2
mkdir -p $o
if [ -n "$tests" ]; then
  timeout -k 10 300 python -u -m pytest $tests -m gpu -v -rf --timeout 100 --timeout-method thread > $o/tests.txt 2>&1
  rc=$?; tail -4 $o/tests.txt; [ $rc -le 1 ] || exit $rc
fi
i=0
for args in "$@"; do
  i=$((i+1))
  timeout -k 10 200 python bench.py --no-cpu-baseline $args > $o/b$i.json 2> $o/b$i.err || { tail -20 $o/b$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$o/b$i.json')); print('$args', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/p$i -o run -- python3 bench.py --no-cpu-baseline $args > $o/p$i.json 2> $o/p$i.err || { tail -20 $o/p$i.err; exit 1; }
  python3 tools/kstats.py $o/p$i/run_kernel_stats.csv | grep -v "k_pack_synth\|k_build_lin\|k_fill_exc\|k_lane_flags\|k_clean_oth\|k_run_inter\|k_sb_flags\|k_fill_halo\|k_build_xlist\|rocprim"
done
