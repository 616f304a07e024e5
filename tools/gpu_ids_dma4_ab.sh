#!/bin/bash
# (The PM_IDS_DMA4 generator form was measured slower and removed again,
# profiles/r06ak_ids_dma4_ab.txt: this script now runs the same code.)
# A/B (round 6): pm_ids_rev's own-column steps fed by one row DMA
# (PM_IDS_DMA4=1, with PM_IDS_BRKSPLIT=0: 121 VGPRs; with the split it
# spills) vs the default (dword DMAs, break split) vs neither; parity tests
# of the DMA4 form first, then the -k 2ids bench under rocprofv3 stats
set -o pipefail
out=gpurun_out/idsdma4
mkdir -p $out
export TMPDIR=/tmp
PM_IDS_DMA4=1 PM_IDS_BRKSPLIT=0 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_ids.py tests/test_gpu_esimple.py tests/test_gpu_wide.py > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
for i in 1 2; do
for cfg in "1 0" "0 1" "0 0"; do
set -- $cfg
PM_IDS_DMA4=$1 PM_IDS_BRKSPLIT=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/d$1b$2.$i -o run -- python3 bench.py --no-cpu-baseline --types ids --steps 10 --warmup 3 > $out/d$1b$2.$i.json 2> $out/d$1b$2.$i.err || { tail -20 $out/d$1b$2.$i.err; exit 1; }
python3 - "$out/d$1b$2.$i" "DMA4=$1 BRKSPLIT=$2 run $i" <<'PY'
import csv, json, sys
d = json.load(open(sys.argv[1] + ".json"))
w = [r for r in csv.DictReader(open(sys.argv[1] + "/run_kernel_stats.csv")) if r["Name"] == "pm_ids_rev"]
print(sys.argv[2], "ms/step", d["ms_per_step"], "pm_ids_rev mean us", round(float(w[0]["AverageNs"]) / 1e3, 1), "hits", d["config"]["hits"])
PY
done
done
