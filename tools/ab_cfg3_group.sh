# cfg 3 on the default build (2-slot home groups) and a 1-slot build (orleans_amd/variants/libgd_g1.so),
# each with and without the compact probe index.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
OUT=gpurun_out/r03_cfg3_group_ab.txt
: > $OUT
for rep in 1 2; do
for v in default g1; do
for cx in 1 0; do
  if [ $v = default ]; then L=orleans_amd/libgraindispatch.so; else L=orleans_amd/variants/libgd_$v.so; fi
  GRAINDISPATCH_LIB=$PWD/$L GD_CX=$cx timeout -k 10 300 python bench.py --workload cfg3 --no-cpu-baseline --no-secondary --latency-batches 0 --steps 20 --warmup 5 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 2; }
  echo "$v GD_CX=$cx $(python -c "import json;d=json.loads(open('gpurun_out/ab.json').readlines()[-1]);print(round(d['value']/1e9,3), d['ms_per_step'], {k: v['ms_per_step'] for k, v in d.get('kernels', {}).items()})")" >> $OUT
done
done
done
