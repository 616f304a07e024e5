#!/bin/bash
# SQ counters of the bench's kernels (k_es_walk among them), one pass per
# counter group.  usage: tools/gpu_pmc_walk.sh <tag> [bench args...]
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > "$out/counters.txt" 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_INSTS_BRANCH" "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > "$out/p$i.json" 2> "$out/p$i.err" || { echo "pass $i failed"; tail -5 "$out/p$i.err"; exit 1; }
done
echo done
