#!/bin/bash
# A/B (round 6): pm_ids_rev with the exception step split by whether some
# lane's word holds a line break (PM_IDS_BRKSPLIT=1, default: the masked
# update only then) vs every exception step masked (0, the round-5 form);
# parity tests first, then the -k 2ids bench under rocprofv3 stats
set -o pipefail
out=gpurun_out/idsbrk
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_ids.py tests/test_gpu_esimple.py tests/test_gpu_wide.py > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
for i in 1 2; do
for v in 1 0; do
PM_IDS_BRKSPLIT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/ids$v.$i -o run -- python3 bench.py --no-cpu-baseline --types ids --steps 10 --warmup 3 > $out/ids$v.$i.json 2> $out/ids$v.$i.err || { tail -20 $out/ids$v.$i.err; exit 1; }
python3 - "$out/ids$v.$i" "PM_IDS_BRKSPLIT=$v run $i" <<'PY'
import csv, json, sys
d = json.load(open(sys.argv[1] + ".json"))
w = [r for r in csv.DictReader(open(sys.argv[1] + "/run_kernel_stats.csv")) if r["Name"] == "pm_ids_rev"]
print(sys.argv[2], "ms/step", d["ms_per_step"], "pm_ids_rev mean us", round(float(w[0]["AverageNs"]) / 1e3, 1), "hits", d["config"]["hits"])
PY
done
done
