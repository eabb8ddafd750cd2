# A/B on the GPU box for the region-mapped owner probe (gd_route_multi): exchange parity tests,
# then bench.py --exchange library (world 1) twice per GD_REGION_PROBE setting.
#   bash tools/ab_region.sh [tests]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ "$1" != "notests" ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_region_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/ab_region_tests.log; exit 1; }
tail -3 gpurun_out/ab_region_tests.log
fi
for i in 1 2; do
for b in 0 1; do
GD_REGION_PROBE=$b timeout -k 10 200 python bench.py --exchange library --steps 100 --warmup 10 --no-cpu-baseline --latency-batches 0 --no-secondary > gpurun_out/ab_region.json 2>gpurun_out/ab_region_err.log || { tail -20 gpurun_out/ab_region_err.log; exit 1; }
python -c "
import json; l=[x for x in open('gpurun_out/ab_region.json') if x.startswith('{')][-1]; d=json.loads(l)
print('GD_REGION_PROBE=$b', round(d['value']/1e9,3), d['ms_per_step'], {k:(v['launches_per_step'],v['ms_per_step']) for k,v in d.get('kernels',{}).items()})"
done; done
