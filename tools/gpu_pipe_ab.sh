set -o pipefail
mkdir -p gpurun_out/pipe
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_ids.py tests/test_gpu_bench_ranks.py > gpurun_out/pipe/tests.txt 2>&1 || { tail -30 gpurun_out/pipe/tests.txt; exit 1; }
tail -2 gpurun_out/pipe/tests.txt
for i in 1 2; do
timeout -k 10 200 python bench.py --types ids --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/pipe/p$i.json 2> gpurun_out/pipe/p$i.err || exit 1
timeout -k 10 200 python bench.py --types ids --steps 10 --warmup 3 --no-cpu-baseline --serial > gpurun_out/pipe/s$i.json 2> gpurun_out/pipe/s$i.err || exit 1
done
for f in p1 s1 p2 s2; do python3 -c "import json;d=json.load(open('gpurun_out/pipe/$f.json'));print('$f',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['config']['hits'],d.get('parity_sample_bit_exact'))"; done
