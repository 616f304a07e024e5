#!/bin/bash
# Round evidence on one GPU box (all under gpurun_out/<tag>):
#   the default bench line (configs[2] 10 Gbp headline + the configs4 and
#   north_star_100gbp extras, CPU baselines and parity samples) and its
#   rocprofv3 --kernel-trace --stats summary; the same for -k 2ids
#   PMC passes (one counter group per run): pm_linear_jit (headline only),
#   FETCH_SIZE / WRITE_SIZE over the default run (all three workloads),
#   pm_ids_rev, and configs[4]'s kernels
#   FETCH_SIZE calibration on known-byte reads (tools/micro/calib_read)
#   configs[0]/[1]/[3] timings with bit-exact checks (tools/config_times.py)
#   a kernel trace of configs[3]'s queries (tools/cfg3_prof.py)
# then: python3 tools/evidence_summary.py gpurun_out/<tag> <round> (host side; also
# writes the steady-state summary, tools/steady_state.py)
# Usage: bash tools/gpu_evidence.sh <tag> [a|b]   (a: benches + headline PMC, b: the rest;
# default both -- two gpurun calls keep each under its time limit)
set -o pipefail
out=gpurun_out/${1:-evidence}
mkdir -p "$out"
export TMPDIR=/tmp
die() { echo "$1 failed"; tail -20 "$2"; exit 1; }
B() { timeout -k 10 "$1" python bench.py "${@:3}" > "$out/$2.json" 2> "$out/$2.err" || die "$2" "$out/$2.err"; cut -c1-200 "$out/$2.json"; }
P() { timeout -k 10 "$1" rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$2" -o run -- python3 bench.py --no-cpu-baseline "${@:3}" > "$out/$2.json" 2> "$out/$2.err" || die "$2" "$out/$2.err"; }
M() { timeout -s KILL "$1" rocprofv3 --pmc $3 --output-format csv -d "$out/$2" -o run -- python3 bench.py --no-cpu-baseline "${@:4}" > "$out/$2.json" 2> "$out/$2.err" || die "pmc $2" "$out/$2.err"; echo "pmc $2 done"; }
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU"
G2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
G3="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
part=${2:-ab}
if [[ $part == *a* ]]; then
B 500 bench --steps 20 --warmup 5
P 500 prof --steps 20 --warmup 5
B 300 bench_ids --types ids --steps 10 --warmup 3
P 300 prof_ids --types ids --steps 10 --warmup 3
M 240 p1 "$G1" --steps 3 --warmup 1 --extras off
M 240 p2 "$G2" --steps 3 --warmup 1 --extras off
M 400 p3 FETCH_SIZE --steps 3 --warmup 1 --extras on
M 400 p4 WRITE_SIZE --steps 3 --warmup 1 --extras on
fi
if [[ $part == *b* ]]; then
M 240 q1 "$G1" --types ids --steps 2 --warmup 1
M 240 q2 "$G2" --types ids --steps 2 --warmup 1
M 240 q3 FETCH_SIZE --types ids --steps 2 --warmup 1
M 240 q4 WRITE_SIZE --types ids --steps 2 --warmup 1
M 240 c1 "$G1" --config 4 --steps 2 --warmup 1
M 240 c2 "$G3" --config 4 --steps 2 --warmup 1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/cal" -o run -- ./tools/micro/calib_read 4096 > "$out/cal.json" 2> "$out/cal.err" || die calibration "$out/cal.err"
timeout -k 10 300 python tools/config_times.py > "$out/configs.json" 2> "$out/configs.err" || die configs "$out/configs.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/cfg3" -o run -- python3 tools/cfg3_prof.py > "$out/cfg3.log" 2>&1 || die cfg3 "$out/cfg3.log"
fi
echo evidence-done
