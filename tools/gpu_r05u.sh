#!/bin/bash
# round 5 experiment: configs[4] report pass with the header check off (timing only)
set -o pipefail
out=gpurun_out/r05u
mkdir -p $out
export TMPDIR=/tmp
PM_EXP_REP_NOHDR=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p1 -o run -- python3 bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline > $out/p1.json 2> $out/p1.err || { tail -20 $out/p1.err; exit 1; }
python3 tools/kstats.py $out/p1/run_kernel_stats.csv | grep -E "rep_|batch_v"
