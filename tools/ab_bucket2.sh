set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_receive.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_b2_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r03_b2_tests.log; exit 1; }
for i in 1 2; do
for b in 0 1; do
GD_BUCKET2=$b timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --latency-batches 0 > gpurun_out/r03_b2_bench_$b_$i.json 2>gpurun_out/r03_b2_bench_err.log || exit 1
python -c "
import json,sys; l=[x for x in open('gpurun_out/r03_b2_bench_$b_$i.json') if x.startswith('{')][-1]; d=json.loads(l)
print('B2=$b', d['value']/1e9, d['ms_per_step'], {k:(v['launches_per_step'],v['ms_per_step']) for k,v in d['kernels'].items()})"
done; done
