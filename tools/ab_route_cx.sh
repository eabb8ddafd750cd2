# A/B of the route kernels with the compact probe index: GD_ROUTE_M, GD_CX_SCALE, GD_ROUTE_NT, GD_CX on
# cfg 2, and GD_CX on the cfg 4 cascade; the fan-out and index parity tests first.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
OUT=gpurun_out/r03_route_cx_ab.txt
: > $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_cx.py tests/test_gpu_fanout.py tests/test_gpu_fanout_multi.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_cx_fan_tests.log 2>&1 || exit 1
for rep in 1 2; do
for cfg in "GD_CX=1" "GD_CX=0" "GD_ROUTE_M=2" "GD_CX_SCALE=2" "GD_ROUTE_NT=1"; do
  env $cfg timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --latency-batches 0 --steps 100 --warmup 10 > gpurun_out/ab.json 2>/dev/null || exit 2
  echo "cfg2 $cfg $(python -c "import json;d=json.loads(open('gpurun_out/ab.json').readlines()[-1]);print(round(d['value']/1e9,3), d['ms_per_step'], d['roofline']['avg_launch_ms'])")" >> $OUT
done
for cfg in "GD_CX=1" "GD_CX=0"; do
  env $cfg timeout -k 10 300 python bench.py --workload cfg4 --no-cpu-baseline > gpurun_out/ab.json 2>/dev/null || exit 3
  echo "cfg4 $cfg $(python -c "import json;d=json.loads(open('gpurun_out/ab.json').readlines()[-1]);print(round(d['value']/1e9,3), d['ms_per_step'], {k: v['ms_per_step'] for k, v in d.get('kernels', {}).items() if 'fan' in k})")" >> $OUT
done
done
