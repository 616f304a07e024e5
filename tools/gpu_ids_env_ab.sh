#!/bin/bash
# A/B (round 6) of a pm_ids_rev generator knob: bash tools/gpu_ids_env_ab.sh <VAR> runs <VAR>=1 (default) vs 0
# (PM_IDS_BRKSPLIT, PM_IDS_M0, ...); parity tests first, then the -k 2ids
# bench under rocprofv3 stats, alternating
set -o pipefail
VAR=${1:?env var}; out=gpurun_out/idsenv_$VAR
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_ids.py tests/test_gpu_esimple.py tests/test_gpu_wide.py > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
for i in 1 2; do
for v in 1 0; do
env "$VAR=$v" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/ids$v.$i -o run -- python3 bench.py --no-cpu-baseline --types ids --steps 10 --warmup 3 > $out/ids$v.$i.json 2> $out/ids$v.$i.err || { tail -20 $out/ids$v.$i.err; exit 1; }
python3 - "$out/ids$v.$i" "$VAR=$v run $i" <<'PY'
import csv, json, sys
d = json.load(open(sys.argv[1] + ".json"))
w = [r for r in csv.DictReader(open(sys.argv[1] + "/run_kernel_stats.csv")) if r["Name"] == "pm_ids_rev"]
print(sys.argv[2], "ms/step", d["ms_per_step"], "pm_ids_rev mean us", round(float(w[0]["AverageNs"]) / 1e3, 1), "hits", d["config"]["hits"])
PY
done
done
