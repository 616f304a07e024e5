#!/bin/bash
# A/B (round 6): configs[4]'s post-verify work (ordered lists' sort, scatter,
# merge, report) on the post stream while the next query scans
# (PM_POST_STREAM=1 / 2) vs on the scan's stream (0, default); parity first.
# The batch half of the knob was measured slower and removed again
# (profiles/r06af_cfg4_post_stream_ab.txt): this script now runs the same
# code three times.
set -o pipefail
out=gpurun_out/postb
mkdir -p $out
PM_POST_STREAM=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_gpu_report.py -k "config4 or batch" > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
for i in 1 2; do
for m in 0 1 2; do
PM_POST_STREAM=$m timeout -k 10 200 python bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline > $out/m$m.$i.json 2> $out/m$m.$i.err || { tail -20 $out/m$m.$i.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/m$m.$i.json'));print('PM_POST_STREAM=$m run $i', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['config']['hits'], d.get('parity_sample_bit_exact'))"
done
done
