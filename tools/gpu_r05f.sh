#!/bin/bash
# round 5: configs[3] latency breakdown (runtime + kernel trace of repeated
# queries) and the per-config times
set -o pipefail
out=gpurun_out/r05f
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/config_times.py > $out/configs.json 2> $out/configs.err || { tail -20 $out/configs.err; exit 1; }
cat $out/configs.json
timeout -k 10 300 rocprofv3 --runtime-trace --kernel-trace --output-format csv -d $out/rt -o run -- python3 tools/cfg3_prof.py > $out/rt.log 2>&1 || { tail -20 $out/rt.log; exit 1; }
grep "query_ms" $out/rt.log
ls $out/rt
