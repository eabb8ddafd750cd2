# A/B on the GPU box for the directory table's slot group (GD_SLOT_GROUP, gd_common.h): the full GPU
# suite on the default build, then bench.py twice per variant library (orleans_amd/variants/).
#   bash tools/ab_slotgroup.sh [notests]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ "$1" != "notests" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_sg_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/ab_sg_tests.log; exit 1; }
tail -3 gpurun_out/ab_sg_tests.log
fi
for i in 1 2; do
for v in default g1 g2 g8; do
if [ $v = default ]; then L=orleans_amd/libgraindispatch.so; else L=orleans_amd/variants/libgd_$v.so; fi
GRAINDISPATCH_LIB=$PWD/$L timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --latency-batches 0 --no-secondary > gpurun_out/ab_sg.json 2>gpurun_out/ab_sg_err.log || { tail -20 gpurun_out/ab_sg_err.log; exit 1; }
python -c "
import json; l=[x for x in open('gpurun_out/ab_sg.json') if x.startswith('{')][-1]; d=json.loads(l)
print('$v', round(d['value']/1e9,3), d['ms_per_step'], {k:v['ms_per_step'] for k,v in d.get('kernels',{}).items()})"
done; done
