#!/bin/bash
# PMC passes over the shape sweep's default shape (short run).
set -o pipefail
tag=${1:-pmc}; shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" "GRBM_GUI_ACTIVE SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o run -- python3 tools/shape_sweep.py 10 TGCTGASTCAGCANW 2 "$@" > "$out/p$i.log" 2> "$out/p$i.err" || { echo "pmc pass $i failed"; tail -5 "$out/p$i.err"; exit 1; }
done
echo done
