#!/bin/bash
# PMC passes (one counter group per run) over the bench, summarized for one
# kernel.  Usage: bash tools/pmc_kernel.sh <tag> <kernel-name-substring> [bench args...]
set -o pipefail
out=gpurun_out/$1; kern=$2; shift 2
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SMEM" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > "$out/p$i.json" 2> "$out/p$i.err" || { echo "pmc pass $i failed"; tail -5 "$out/p$i.err"; exit 1; }
done
python3 tools/pmc_summary.py "$out" "$kern" > "$out/pmc_summary.txt" 2>&1
cat "$out/pmc_summary.txt"
