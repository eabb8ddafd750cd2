# cfg 3 (64M Zipf(1.1) messages over 100M grains, one GPU) with and without the compact probe index.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
OUT=gpurun_out/r03_cfg3_cx_ab.txt
: > $OUT
for rep in 1 2; do
for cfg in "GD_CX=1" "GD_CX=0"; do
  env $cfg timeout -k 10 300 python bench.py --workload cfg3 --no-cpu-baseline --no-secondary --latency-batches 0 --steps 20 --warmup 5 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 2; }
  echo "$cfg $(python -c "import json;d=json.loads(open('gpurun_out/ab.json').readlines()[-1]);print(round(d['value']/1e9,3), d['ms_per_step'], {k: v['ms_per_step'] for k, v in d.get('kernels', {}).items()})")" >> $OUT
done
done
