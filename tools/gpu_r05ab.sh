#!/bin/bash
# round 5: zero-copy hand-over of the hit list to torch (bench collect) --
# its test, the multi-rank bench tests, configs[2] / configs[4] benches
set -o pipefail
out=gpurun_out/r05ab
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_zero_copy.py tests/test_gpu_bench_ranks.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/t.log 2>&1 || { tail -40 $out/t.log; exit 1; }
tail -2 $out/t.log
for r in 1 2; do
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/c2_$r.json 2> $out/c2_$r.err || { tail -20 $out/c2_$r.err; exit 1; }
timeout -k 10 300 python3 bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline > $out/c4_$r.json 2> $out/c4_$r.err || { tail -20 $out/c4_$r.err; exit 1; }
echo "run $r cfg2 $(python3 -c "import json;print(json.load(open('$out/c2_$r.json'))['ms_per_step'])") cfg4 $(python3 -c "import json;print(json.load(open('$out/c4_$r.json'))['ms_per_step'])")"
done
