#!/bin/bash
# Same-box sweep of the specialized kernel's workgroup split (PM_JIT_SPLIT)
# and resident workgroups per CU (PM_JIT_WAVES) on the default bench line.
# usage: bash tools/gpu_split.sh <tag>
set -o pipefail
o=gpurun_out/$1
mkdir -p $o
run() {
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py > $o/$name.json 2> $o/$name.err || { tail -20 $o/$name.err; exit 1; }
  tail -1 $o/$name.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$name', d['value'], d['ms_per_step'], r['achieved'], r['frac'])"
}
run def1 PM_X=0
run s4 PM_JIT_SPLIT=4
run s16 PM_JIT_SPLIT=16
run s32 PM_JIT_SPLIT=32
run def2 PM_X=0
run s12 PM_JIT_SPLIT=12
run s6 PM_JIT_SPLIT=6
run w3 PM_JIT_WAVES=3
run def3 PM_X=0
