set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_cx.py tests/test_gpu_parity.py tests/test_host_cpp.py tests/test_gpu_cache_keyext.py tests/test_gpu_cache.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_cx_tests.log 2>&1 || exit 1
for cx in 1 0 1 0; do
  GD_CX=$cx timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > gpurun_out/r03_cx_bench_$cx.json 2>/dev/null || exit 2
  echo "GD_CX=$cx $(python -c "import json;d=json.loads(open('gpurun_out/r03_cx_bench_$cx.json').readlines()[-1]);print(d['value']/1e9, d['ms_per_step'], d['roofline']['avg_launch_ms'])")" >> gpurun_out/r03_cx_ab.txt
done
