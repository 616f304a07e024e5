#!/bin/bash
# round-4 GPU check: the -k ids parity tests, the whole -m gpu suite, the
# ids bench line and its PMC passes (FETCH_SIZE against the algorithmic bytes).
set -o pipefail
tag=${1:-r04}; out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ids.py -m gpu -x -q --timeout 200 --timeout-method thread > "$out/ids.txt" 2>&1 || { tail -30 "$out/ids.txt"; exit 1; }
tail -1 "$out/ids.txt"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > "$out/all.txt" 2>&1
rc=$?; tail -6 "$out/all.txt"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --types ids --steps 5 --warmup 2 --no-cpu-baseline > "$out/bench_ids.json" 2> "$out/bench_ids.err" || { tail -20 "$out/bench_ids.err"; exit 1; }
cut -c1-600 "$out/bench_ids.json"
bash tools/pmc_kernel.sh "$tag/pmc" pm_ids --types ids
