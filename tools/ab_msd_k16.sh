# The two-level bucketing: the MSD pass writing the range-local keys as u16 (GD_MSD_K16=1) or u32:
# the parity tests, then cfg 2 A/B.  (Earlier: GD_MSD_TILE 16384 vs 8192, GD_MSD_EARLY 0 vs 1.)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
OUT=gpurun_out/r03_msd_k16_ab.txt
: > $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_msd.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_msd_k16_tests.log 2>&1 || { tail -40 gpurun_out/r03_msd_k16_tests.log; exit 1; }
for rep in 1 2; do
for m in "GD_MSD_K16=0" "GD_MSD_K16=1"; do
  env GD_MSD=2 $m timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --latency-batches 0 --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 2; }
  echo "cfg2 GD_MSD=2 $m $(python -c "import json;d=json.loads(open('gpurun_out/ab.json').readlines()[-1]);print(round(d['value']/1e9,3), d['ms_per_step'], {k: v['ms_per_step'] for k, v in d.get('kernels', {}).items()})")" >> $OUT
done; done
