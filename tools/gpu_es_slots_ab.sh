#!/bin/bash
# A/B (round 6): k_es_walk with the esimple slots staged in LDS
# (PM_ES_SLOTS_LDS=1, default) vs read from global memory (0): the walk's
# kernel time in rocprofv3 stats over the -k 2ids bench and the headline
set -o pipefail
out=gpurun_out/esslots
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_esimple.py tests/test_gpu_ids.py > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
for i in 1 2; do
for v in 1 0; do
for w in ids head; do
args="--types ids --steps 10 --warmup 3"; [ $w = head ] && args="--extras off --steps 20 --warmup 5"
PM_ES_SLOTS_LDS=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$w$v.$i -o run -- python3 bench.py --no-cpu-baseline $args > $out/$w$v.$i.json 2> $out/$w$v.$i.err || { tail -20 $out/$w$v.$i.err; exit 1; }
python3 - "$out/$w$v.$i" "$w PM_ES_SLOTS_LDS=$v run $i" <<'PY'
import csv, json, sys
d = json.load(open(sys.argv[1] + ".json"))
w = [r for r in csv.DictReader(open(sys.argv[1] + "/run_kernel_stats.csv")) if "k_es_walk" in r["Name"]]
print(sys.argv[2], "ms/step", d["ms_per_step"], "k_es_walk mean us", round(float(w[0]["AverageNs"]) / 1e3, 1) if w else None, "hits", d["config"]["hits"])
PY
done
done
done
