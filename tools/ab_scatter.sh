# A/B on the GPU box: bucketing parity tests, then bench.py twice per setting of one switch
#   bash tools/ab_scatter.sh VAR "A B"
set -o pipefail
cd $GRAFT_REPO_ROOT
VAR=$1; VALS=$2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bucket2.py tests/test_gpu_receive.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/ab_tests.log; exit 1; }
for i in 1 2; do
for b in $VALS; do
env $VAR=$b timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --latency-batches 0 --no-secondary > gpurun_out/ab_bench.json 2>gpurun_out/ab_bench_err.log || { tail -20 gpurun_out/ab_bench_err.log; exit 1; }
python -c "
import json; l=[x for x in open('gpurun_out/ab_bench.json') if x.startswith('{')][-1]; d=json.loads(l)
print('$VAR=$b', round(d['value']/1e9,3), d['ms_per_step'], {k:(v['launches_per_step'],v['ms_per_step']) for k,v in d['kernels'].items()})"
done; done
