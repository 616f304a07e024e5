#!/bin/bash
# k_es_walk experiments: PM_ES_MODE 0 (full), 1 (setup only), 2 (no verify)
tag=$1
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for t in s ids; do
  for mode in 0 1 2; do
    PM_ES_MODE=$mode timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/${t}_m$mode" -o run -- python3 tools/es_probe.py $t > "$out/${t}_m$mode.log" 2>&1 || { echo "fail $t $mode"; tail -5 "$out/${t}_m$mode.log"; exit 1; }
  done
done
for f in "$out"/*/run_kernel_stats.csv; do echo "$f"; grep -E "k_es_walk|k_es_heads" "$f" | cut -c1-200; done
