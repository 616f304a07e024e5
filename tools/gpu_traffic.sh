#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate) for the bench kernel + a 4 GiB calibration read.
set -o pipefail
out=gpurun_out/${1:-traffic}
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$out/b$i" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$out/b$i.json" 2> "$out/b$i.err" || { echo "bench pmc $grp failed"; tail -5 "$out/b$i.err"; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$out/c$i" -o run -- python3 tools/calib_fetch.py > "$out/c$i.log" 2> "$out/c$i.err" || { echo "calib pmc $grp failed"; tail -5 "$out/c$i.err"; exit 1; }
done
echo done
