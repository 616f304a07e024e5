#!/bin/bash
# Round evidence on one GPU box (all under gpurun_out/<tag>):
#   bench lines: configs[2] default (+ CPU baseline), 100 Gbp, -k 2ids, configs[4]
#   rocprofv3 --kernel-trace --stats summaries of the same commands
#   PMC passes (one counter group per run) on pm_linear_jit and pm_ids_rev
#   FETCH_SIZE calibration on known-byte reads (tools/micro/calib_read)
#   configs[0]/[1]/[3] timings with bit-exact checks (tools/config_times.py)
# then: python3 tools/evidence_summary.py gpurun_out/<tag> <round> (host side)
# Usage: bash tools/gpu_evidence_a.sh <tag>  (bench lines + rocprof stats; part B: PMC, calibration, configs)
set -o pipefail
out=gpurun_out/${1:-evidence}
mkdir -p "$out"
export TMPDIR=/tmp
die() { echo "$1 failed"; tail -20 "$2"; exit 1; }
B() { timeout -k 10 "$1" python bench.py "${@:3}" > "$out/$2.json" 2> "$out/$2.err" || die "$2" "$out/$2.err"; cut -c1-200 "$out/$2.json"; }
P() { timeout -k 10 "$1" rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$2" -o run -- python3 bench.py --no-cpu-baseline "${@:3}" > "$out/$2.json" 2> "$out/$2.err" || die "$2" "$out/$2.err"; }
B 300 bench --steps 20 --warmup 5
P 300 prof --steps 20 --warmup 5
B 400 bench100 --gbp 100 --steps 10 --warmup 3
P 400 prof100 --gbp 100 --steps 10 --warmup 3
B 300 bench_ids --types ids --steps 10 --warmup 3
P 300 prof_ids --types ids --steps 10 --warmup 3
B 400 bench_cfg4 --config 4 --steps 3 --warmup 1 --no-cpu-baseline
P 400 prof_cfg4 --config 4 --steps 3 --warmup 1
echo evidence-a-done
