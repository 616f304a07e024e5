#!/bin/bash
# Round evidence on one GPU box: bench lines (10 Gbp default, 100 Gbp), the
# rocprofv3 kernel-trace summaries of the same commands, PMC passes on the
# hot kernel (one counter group per run) and the FETCH_SIZE calibration.
# Usage: bash tools/gpu_evidence.sh <tag>
set -o pipefail
out=gpurun_out/${1:-evidence}
mkdir -p "$out"
export TMPDIR=/tmp
run() { echo "== $*" >&2; "$@"; }
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err" || { echo "bench failed"; tail -20 "$out/bench.err"; exit 1; }
cat "$out/bench.json"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$out/bench_prof.json" 2> "$out/bench_prof.err" || { echo "rocprof failed"; tail -20 "$out/bench_prof.err"; exit 1; }
cat "$out/bench_prof.json"
timeout -k 10 400 python bench.py --gbp 100 --steps 10 --warmup 3 > "$out/bench100.json" 2> "$out/bench100.err" || { echo "bench 100 failed"; tail -20 "$out/bench100.err"; exit 1; }
cat "$out/bench100.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof100" -o run -- python3 bench.py --gbp 100 --steps 10 --warmup 3 --no-cpu-baseline > "$out/bench100_prof.json" 2> "$out/bench100_prof.err" || { echo "rocprof 100 failed"; tail -20 "$out/bench100_prof.err"; exit 1; }
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$out/p$i.json" 2> "$out/p$i.err" || { echo "pmc pass $i failed"; tail -5 "$out/p$i.err"; exit 1; }
done
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/cal" -o run -- ./tools/micro/calib_read 4096 > "$out/cal.json" 2> "$out/cal.err" || { echo "calibration failed"; tail -5 "$out/cal.err"; exit 1; }
python3 tools/pmc_summary.py "$out" pm_linear_jit > "$out/pmc_summary.txt" 2>&1
cat "$out/pmc_summary.txt"
echo evidence-done
