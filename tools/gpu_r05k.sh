#!/bin/bash
# round 5: block radix sort of mid/big bins, k_rep_walk neighbour fast path,
# pm_ids_rev keeps the warm-up words in LDS, k_es_walk 4-wave blocks -- the GPU suite, configs[4] and
# -k 2ids benches (keep on / off) + kernel traces
set -o pipefail
out=gpurun_out/r05k
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/t.log 2>&1 || { tail -40 $out/t.log; exit 1; }
tail -2 $out/t.log
timeout -k 10 300 python3 bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline > $out/bench4.json 2> $out/bench4.err || { tail -20 $out/bench4.err; exit 1; }
cut -c1-300 $out/bench4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof4 -o run -- python3 bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline > $out/prof4.json 2> $out/prof4.err || { tail -20 $out/prof4.err; exit 1; }
python3 tools/kstats.py $out/prof4/run_kernel_stats.csv | head -16
for v in "1 1" "0 1" "1 3"; do
  set -- $v
  PM_IDS_KEEP=$1 PM_ES_OCC=$2 timeout -k 10 300 python3 bench.py --types ids --steps 10 --warmup 3 --no-cpu-baseline > $out/ids$1$2.json 2> $out/ids$1$2.err || { tail -20 $out/ids$1$2.err; exit 1; }
  echo "keep=$1 es_occ=$2"; cut -c1-300 $out/ids$1$2.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/profids -o run -- python3 bench.py --types ids --steps 10 --warmup 3 --no-cpu-baseline > $out/profids.json 2> $out/profids.err || { tail -20 $out/profids.err; exit 1; }
python3 tools/kstats.py $out/profids/run_kernel_stats.csv | head -12
