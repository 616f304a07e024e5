#!/bin/bash
# round 5: k_rep_walk candidates per thread (PM_REP_RW 2 / 4 / 8) on
# configs[4] and configs[2], alternating
set -o pipefail
out=gpurun_out/r05aa
mkdir -p $out
export TMPDIR=/tmp
for r in 1 2; do
for w in 4 8 2; do
PM_REP_RW=$w timeout -k 10 300 python3 bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline > $out/c4_${w}_$r.json 2> $out/c4_${w}_$r.err || { tail -20 $out/c4_${w}_$r.err; exit 1; }
PM_REP_RW=$w timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/c2_${w}_$r.json 2> $out/c2_${w}_$r.err || { tail -20 $out/c2_${w}_$r.err; exit 1; }
echo "rw $w run $r cfg4 $(python3 -c "import json;print(json.load(open('$out/c4_${w}_$r.json'))['ms_per_step'])") cfg2 $(python3 -c "import json;print(json.load(open('$out/c2_${w}_$r.json'))['ms_per_step'])")"
done
done
PM_REP_RW=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p8 -o run -- python3 bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline > $out/p8.json 2> $out/p8.err || { tail -20 $out/p8.err; exit 1; }
python3 tools/kstats.py $out/p8/run_kernel_stats.csv | grep rep_
