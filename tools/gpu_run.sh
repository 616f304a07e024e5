#!/bin/bash
# One GPU call, several steps, each under its own time limit; the first step
# that fails for a reason other than test failures (timeout, abort, crash)
# ends the call.  Outputs under gpurun_out/<tag>/.
#   bash tools/gpu_run.sh <tag> <step> [<step> ...]
# steps:
#   test=<name>:<pytest args>     python -m pytest <args> (rc 0/1 go on)
#   bench=<name>:<bench args>     python bench.py <args> > <name>.json
#   prof=<name>:<bench args>      rocprofv3 --kernel-trace --stats of bench.py
#   pmc=<name>:<counters>:<bench args>   one rocprofv3 --pmc pass of bench.py
#   py=<name>:<script args>       python <script args> > <name>.out
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for s in "$@"; do
    kind=${s%%=*}; rest=${s#*=}; name=${rest%%:*}; args=${rest#*:}
    case $kind in
        test)  timeout -k 10 900 python -u -m pytest $args --timeout 240 --timeout-method thread > "$out/$name.txt" 2>&1; rc=$?
               tail -3 "$out/$name.txt"; [ $rc -le 1 ] || { echo "$name rc=$rc"; exit $rc; } ;;
        bench) timeout -k 10 600 python bench.py $args > "$out/$name.json" 2> "$out/$name.err"; rc=$?
               cut -c1-300 "$out/$name.json"; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -20 "$out/$name.err"; exit $rc; } ;;
        prof)  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$name" -o run -- python3 bench.py $args > "$out/$name.json" 2> "$out/$name.err"; rc=$?
               [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -20 "$out/$name.err"; exit $rc; } ;;
        pmc)   ctr=${args%%:*}; bargs=${args#*:}
               timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d "$out/$name" -o run -- python3 bench.py $bargs > "$out/$name.json" 2> "$out/$name.err"; rc=$?
               [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -20 "$out/$name.err"; exit $rc; } ;;
        py)    timeout -k 10 600 python $args > "$out/$name.out" 2> "$out/$name.err"; rc=$?
               tail -5 "$out/$name.out"; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -20 "$out/$name.err"; exit $rc; } ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
    echo "$name done rc=$rc"
done
echo all-done
