# The two-level bucketing's MSD histogram: 1, 2 or 4 8K-item tiles a workgroup (GD_MSD_HTPB), cfg 2;
# the MSD parity tests first.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
OUT=gpurun_out/r03_msd_htpb_ab.txt
: > $OUT
for t in 1 2; do
GD_MSD_HTPB=$t timeout -k 10 400 python -u -m pytest tests/test_gpu_msd.py -x -q --timeout 200 --timeout-method thread -k "uniform or measured" > gpurun_out/r03_msd_htpb_tests.log 2>&1 || { tail -40 gpurun_out/r03_msd_htpb_tests.log; exit 1; }
done
for rep in 1 2; do
for t in 4 2 1; do
  env GD_MSD=2 GD_MSD_HTPB=$t timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --latency-batches 0 --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 2; }
  echo "cfg2 GD_MSD=2 GD_MSD_HTPB=$t $(python -c "import json;d=json.loads(open('gpurun_out/ab.json').readlines()[-1]);print(round(d['value']/1e9,3), d['ms_per_step'], {k: v['ms_per_step'] for k, v in d.get('kernels', {}).items()})")" >> $OUT
done; done
