#!/bin/bash
# round 5: the whole GPU suite on the committed tree
set -o pipefail
out=gpurun_out/r05q
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/t.log 2>&1 || { tail -40 $out/t.log; exit 1; }
tail -2 $out/t.log
timeout -k 10 300 python3 bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline > $out/bench4.json 2> $out/bench4.err || { tail -20 $out/bench4.err; exit 1; }
cut -c1-300 $out/bench4.json
