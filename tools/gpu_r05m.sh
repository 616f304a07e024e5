#!/bin/bash
# round 5: configs[4] PMC passes (one counter group per run) for the batch
# kernels: k_batch_scan, k_batch_verify, k_others_batch, the report pass
set -o pipefail
out=gpurun_out/r05m
mkdir -p $out
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o run -- python3 bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > "$out/p$i.json" 2> "$out/p$i.err" || { echo "pmc pass $i failed"; tail -5 "$out/p$i.err"; exit 1; }
done
for k in k_batch_scan k_batch_verify k_others_batch k_rep_walk; do
  echo "== $k"; python3 tools/pmc_summary.py "$out" "$k"
done
