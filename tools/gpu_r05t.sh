#!/bin/bash
# round 5: the batch verify looks codes up in an LDS hash table; the
# extended walk's simple window scanner reads a step ahead -- walk and batch
# tests, configs latency, configs[4] A/B (PM_BATCH_HASH=0: the code array)
set -o pipefail
out=gpurun_out/r05t
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_extended.py tests/test_gpu_eextended.py tests/test_configs_gpu.py tests/test_gpu_report.py tests/test_gpu_regions.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/t.log 2>&1 || { tail -40 $out/t.log; exit 1; }
tail -2 $out/t.log
timeout -k 10 300 python3 tools/config_times.py > $out/configs.json 2> $out/configs.err || { tail -20 $out/configs.err; exit 1; }
cat $out/configs.json
for h in 1 0 1 0; do
  PM_BATCH_HASH=$h timeout -k 10 300 python3 bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline > $out/b4h$h.json 2> $out/b4h$h.err || { tail -20 $out/b4h$h.err; exit 1; }
  echo "hash=$h"; cut -c1-200 $out/b4h$h.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof4 -o run -- python3 bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline > $out/prof4.json 2> $out/prof4.err || { tail -20 $out/prof4.err; exit 1; }
python3 tools/kstats.py $out/prof4/run_kernel_stats.csv | head -8
