#!/bin/bash
# round 5: ordered lists: stable scatter by pattern vs radix (PM_BATCH_SCATTER=0) --
# batch tests, configs[4] x3, kernel stats
set -o pipefail
out=gpurun_out/r05ah
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_report.py tests/test_gpu_parity.py tests/test_gpu_p5.py -m gpu -x -q --timeout 300 --timeout-method thread -k "batch or config4" > $out/t.log 2>&1 || { tail -40 $out/t.log; exit 1; }
tail -2 $out/t.log
for r in 1 2; do
timeout -k 10 300 python3 bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline > $out/on_$r.json 2> $out/on_$r.err || { tail -20 $out/on_$r.err; exit 1; }
PM_BATCH_SCATTER=0 timeout -k 10 300 python3 bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline > $out/off_$r.json 2> $out/off_$r.err || { tail -20 $out/off_$r.err; exit 1; }
echo "scatter on $(python3 -c "import json;print(json.load(open('$out/on_$r.json'))['ms_per_step'])") off $(python3 -c "import json;print(json.load(open('$out/off_$r.json'))['ms_per_step'])")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof4 -o run -- python3 bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline > $out/prof4.json 2> $out/prof4.err || { tail -20 $out/prof4.err; exit 1; }
python3 tools/kstats.py $out/prof4/run_kernel_stats.csv > $out/kstats.txt; grep -E "rep_|batch|scatter|rocprim" $out/kstats.txt | cut -c1-110
