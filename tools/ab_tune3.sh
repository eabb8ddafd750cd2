# Probe variants (GD_CX 1 measured / 2 index group reads / 3 index slot reads / 0 directory), cfg 2 and
# cfg 3; index parity tests first.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
OUT=gpurun_out/r03_tune3_ab.txt
: > $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_cx.py tests/test_gpu_parity.py tests/test_gpu_multi.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_tune3_tests.log 2>&1 || { tail -30 gpurun_out/r03_tune3_tests.log; exit 1; }
for w in cfg2 cfg3; do
for rep in 1 2; do
for cx in 1 2 3 0; do
  GD_CX=$cx timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-secondary --latency-batches 0 --steps 40 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 2; }
  echo "$w GD_CX=$cx $(python -c "import json;d=json.loads(open('gpurun_out/ab.json').readlines()[-1]);print(round(d['value']/1e9,3), d['ms_per_step'], {k: v['ms_per_step'] for k, v in d.get('kernels', {}).items() if k == 'k_route'})")" >> $OUT
done; done; done
