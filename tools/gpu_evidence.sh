#!/bin/bash
# Round evidence on one GPU box (all under gpurun_out/<tag>):
#   bench lines: configs[2] default (+ CPU baseline), 100 Gbp, -k 2ids, configs[4]
#   rocprofv3 --kernel-trace --stats summaries of the same commands
#   PMC passes (one counter group per run) on pm_linear_jit and pm_ids_rev
#   FETCH_SIZE calibration on known-byte reads (tools/micro/calib_read)
#   configs[0]/[1]/[3] timings with bit-exact checks (tools/config_times.py)
#   a kernel trace of configs[3]'s queries (tools/cfg3_prof.py)
# then: python3 tools/evidence_summary.py gpurun_out/<tag> <round> (host side)
# Usage: bash tools/gpu_evidence.sh <tag>
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
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$out/p$i.json" 2> "$out/p$i.err" || die "pmc pass $i" "$out/p$i.err"
  timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d "$out/q$i" -o run -- python3 bench.py --types ids --steps 2 --warmup 1 --no-cpu-baseline > "$out/q$i.json" 2> "$out/q$i.err" || die "ids pmc pass $i" "$out/q$i.err"
done
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d "$out/c$i" -o run -- python3 bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > "$out/c$i.json" 2> "$out/c$i.err" || die "batch pmc pass $i" "$out/c$i.err"
done
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/cal" -o run -- ./tools/micro/calib_read 4096 > "$out/cal.json" 2> "$out/cal.err" || die calibration "$out/cal.err"
timeout -k 10 300 python tools/config_times.py > "$out/configs.json" 2> "$out/configs.err" || die configs "$out/configs.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/cfg3" -o run -- python3 tools/cfg3_prof.py > "$out/cfg3.log" 2>&1 || die cfg3 "$out/cfg3.log"
echo evidence-done
