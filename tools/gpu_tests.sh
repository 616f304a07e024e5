#!/bin/bash
# GPU test recipe: the given test selection first, then the whole -m gpu suite.
# Test failures (pytest rc 1) go on to the next step; a timeout, abort or
# crash (any other rc) ends the call there.
# usage: tools/gpu_tests.sh <tag> <first pytest target...>
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
run() {   # name, seconds, pytest args...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" python -u -m pytest "$@" --timeout 240 --timeout-method thread > "$out/$name.txt" 2>&1
    local rc=$?
    echo "$name rc=$rc" >> "$out/status.txt"
    tail -3 "$out/$name.txt"
    [ $rc -eq 0 ] || [ $rc -eq 1 ]
}
run first 400 -v "$@" && run all 1000 tests -m gpu -q -rf
