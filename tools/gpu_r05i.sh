#!/bin/bash
# round 5: walks templated on scanner / row count, k_nfa_rev's BYTE text in
# 16-byte groups -- the whole GPU suite, configs latency, configs[3] trace
set -o pipefail
out=gpurun_out/r05i
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/t.log 2>&1 || { tail -40 $out/t.log; exit 1; }
tail -3 $out/t.log
timeout -k 10 300 python3 tools/config_times.py > $out/configs.json 2> $out/configs.err || { tail -20 $out/configs.err; exit 1; }
cat $out/configs.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o run -- python3 tools/cfg3_prof.py > $out/kt.log 2>&1 || { tail -20 $out/kt.log; exit 1; }
grep "query_ms" $out/kt.log
