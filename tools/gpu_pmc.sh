#!/bin/bash
# Separate rocprofv3 --pmc passes (one counter group per pass) over a short bench run.
set -o pipefail
tag=${1:-pmc}; shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" "GRBM_GUI_ACTIVE SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > "$out/p$i.json" 2> "$out/p$i.err" || { echo "pmc pass $i failed"; tail -5 "$out/p$i.err"; exit 1; }
done
echo done
