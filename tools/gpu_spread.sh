#!/bin/bash
# Run-to-run spread of the default configs[2] bench line on one box:
# five back-to-back runs (no CPU baseline), one summary line each.
set -o pipefail
out=gpurun_out/spread
mkdir -p $out
for i in 1 2 3 4 5; do
    timeout -k 10 180 python bench.py --no-cpu-baseline > $out/b$i.json 2> $out/b$i.err || { tail -5 $out/b$i.err; exit 1; }
    python3 -c "import json,sys; a=json.load(open(sys.argv[1])); r=a['roofline']; print('run %s: %.1f Gbases/s, %.4f ms/step, kernel mean %.4f ms, frac %.4f' % (sys.argv[2], a['value'], a['ms_per_step'], r['kernel_ms'], r['frac']))" $out/b$i.json $i | tee -a $out/spread.txt
done
