#!/bin/bash
# pm_ids_rev A/B on the `-k 2ids` bench: builds and lane-column lengths,
# alternating.  Usage: bash tools/gpu_idsab.sh <old .so> <mode>...
# (mode: old | <PM_IDS_WPL value>).  Ends with a kernel trace of each mode.
set -o pipefail
OUT=gpurun_out/idsab
mkdir -p $OUT
old=$1; shift
run() {   # mode, out file, bench args...
    local m=$1 f=$2; shift 2
    if [ $m = old ]; then export PM_LIB_AB=$old; unset PM_IDS_WPL; else unset PM_LIB_AB; export PM_IDS_WPL=$m; fi
    timeout -k 10 240 "$@" > $f 2> $f.err
}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_ids.py tests/test_gpu_esimple.py > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
for i in 1 2; do
    for m in "$@"; do
        run $m $OUT/bench_$m$i.json python bench.py --types ids --steps 10 --warmup 3 --no-cpu-baseline \
            || { tail -20 $OUT/bench_$m$i.json.err; exit 1; }
        echo "$m $(python -c "import json; d=json.loads(open('$OUT/bench_$m$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
    done
done
for m in "$@"; do
    run $m $OUT/prof_$m.log rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$m -o ids -- \
        python3 bench.py --types ids --steps 5 --warmup 2 --no-cpu-baseline || { tail -5 $OUT/prof_$m.log.err; exit 1; }
    f=$(find $OUT/prof_$m -name 'ids_kernel_stats.csv' | head -1)
    [ -n "$f" ] && grep -E "pm_ids_rev|Name" "$f" | cut -c1-200
done
exit 0
