#!/bin/bash
# A/B (round 6) of a pm_linear_jit generator knob: bash tools/gpu_jit_env_ab.sh <VAR>
# runs <VAR>=1 (default) vs 0 -- parity tests first, then the headline
# (configs[2], extras off) under rocprofv3 stats, alternating
set -o pipefail
VAR=${1:?env var}; out=gpurun_out/jitenv_$VAR
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_jit_shift.py tests/test_gpu_parity.py tests/test_gpu_graded.py > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
for i in 1 2 3; do
for v in 1 0; do
env "$VAR=$v" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/h$v.$i -o run -- python3 bench.py --no-cpu-baseline --extras off --steps 20 --warmup 5 > $out/h$v.$i.json 2> $out/h$v.$i.err || { tail -20 $out/h$v.$i.err; exit 1; }
python3 - "$out/h$v.$i" "$VAR=$v run $i" <<'PY'
import csv, json, sys
d = json.load(open(sys.argv[1] + ".json"))
w = [r for r in csv.DictReader(open(sys.argv[1] + "/run_kernel_stats.csv")) if r["Name"] == "pm_linear_jit"]
print(sys.argv[2], "Gbases/s", d["value"], "ms/step", d["ms_per_step"], "kernel_ms (HIP events)", d["roofline"]["kernel_ms"],
      "rocprof mean us", round(float(w[0]["AverageNs"]) / 1e3, 1), "hits", d["config"]["hits"])
PY
done
done
