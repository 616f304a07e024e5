#!/bin/bash
# Probes: configs[2] with the exception pass concurrent to the scan, and PMC
# passes on k_batch_verify (configs[4]).
# usage: bash tools/gpu_probe.sh <tag>
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/$1
mkdir -p $o
for v in 0 1; do
  PM_EXC_CONCURRENT=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $o/bench2_conc$v.json 2> $o/bench2_conc$v.err || exit 1
  cut -c1-160 $o/bench2_conc$v.json
  grep -o '"kernel_ms": [0-9.]*' $o/bench2_conc$v.json
done
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d "$o/p$i" -o run -- python3 bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > "$o/p$i.json" 2> "$o/p$i.err" || { echo "pmc pass $i failed"; tail -5 "$o/p$i.err"; exit 1; }
done
python3 tools/pmc_summary.py "$o" k_batch_verify
