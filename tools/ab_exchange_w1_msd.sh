# World-1 library exchange pipeline (gd_route_multi_device, RCCL self send/recv) with the two-level
# bucketing (default, measured choice) and with the LSD passes (GD_MSD=0).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
OUT=gpurun_out/r03_exchange_w1_msd_ab.txt
: > $OUT
for rep in 1 2; do
for cfg in "GD_MSD=1" "GD_MSD=0"; do
  env $cfg timeout -k 10 200 python bench.py --exchange library --no-cpu-baseline --no-secondary --latency-batches 0 --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 2; }
  echo "$cfg $(python -c "import json;d=json.loads(open('gpurun_out/ab.json').readlines()[-1]);print(round(d['value']/1e9,3), d['ms_per_step'], d['exchange'][:40], {k: v['ms_per_step'] for k, v in d.get('kernels', {}).items()})")" >> $OUT
done
done
