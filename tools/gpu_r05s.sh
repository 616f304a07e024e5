#!/bin/bash
# round 5: the extended walk (k = 0) templated on scanner and words, loads a step ahead
# (prefix scanner, checkMatch1 phases) -- walk tests, configs latency, trace
set -o pipefail
out=gpurun_out/r05s
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_extended.py tests/test_gpu_eextended.py tests/test_gpu_regular.py tests/test_configs_gpu.py tests/test_service_gpu.py tests/test_gpu_regions.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/t.log 2>&1 || { tail -40 $out/t.log; exit 1; }
tail -2 $out/t.log
timeout -k 10 300 python3 tools/config_times.py > $out/configs.json 2> $out/configs.err || { tail -20 $out/configs.err; exit 1; }
cat $out/configs.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o run -- python3 tools/cfg3_prof.py > $out/kt.log 2>&1 || { tail -20 $out/kt.log; exit 1; }
grep "query_ms" $out/kt.log
python3 tools/kstats.py $out/kt/run_kernel_stats.csv | head -6
