# cfg 4 cascade and cfg 2 with the probe choice measured per size class (GD_CX=1), forced (2), off (0).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
OUT=gpurun_out/r03_cfg4_tune_ab.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_cx.py tests/test_gpu_fanout.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_cx_tests2.log 2>&1 || exit 1
: > $OUT
for rep in 1 2; do
for cx in 1 2 0; do
  GD_CX=$cx timeout -k 10 300 python bench.py --workload cfg4 --no-cpu-baseline > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 2; }
  echo "cfg4 GD_CX=$cx $(python -c "import json;d=json.loads(open('gpurun_out/ab.json').readlines()[-1]);print(round(d['value']/1e9,3), d['ms_per_step'], {k: v['ms_per_step'] for k, v in d.get('kernels', {}).items() if 'fan_route' in k})")" >> $OUT
done
GD_CX=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --latency-batches 0 --steps 40 --warmup 8 > gpurun_out/ab.json 2>gpurun_out/ab.err || exit 3
echo "cfg2 GD_CX=1 $(python -c "import json;d=json.loads(open('gpurun_out/ab.json').readlines()[-1]);print(round(d['value']/1e9,3), d['ms_per_step'])")" >> $OUT
done
