#!/bin/bash
# round 5: the regular engine's GPU walk against the oracle, then the
# engines that share the report plumbing (extended, eextended, esimple)
set -o pipefail
out=gpurun_out/r05b
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_regular.py -m gpu -v --timeout 300 --timeout-method thread > $out/t_regular.log 2>&1
rc=$?
tail -25 $out/t_regular.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_extended.py tests/test_gpu_eextended.py tests/test_gpu_esimple.py tests/test_configs_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $out/t_others.log 2>&1
rc2=$?
tail -8 $out/t_others.log
exit $(( rc > rc2 ? rc : rc2 ))
