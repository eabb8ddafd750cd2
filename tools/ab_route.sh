#!/bin/bash
# A/B of the cfg 2 step against an older build (orleans_amd/variants/libgd_r05.so): interleaved rounds,
# one compact line each (value, ms a step, k_route's event-timed launch).
set -o pipefail
for r in 1 2 3; do
  for lib in "" "orleans_amd/variants/libgd_r05.so"; do
    if [ -n "$lib" ]; then export GRAINDISPATCH_LIB=$lib; else unset GRAINDISPATCH_LIB; fi
    timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-secondary --no-cpu-baseline --latency-batches 0 \
      --full-out gpurun_out/ab_full.json > gpurun_out/ab_one.log 2>&1 || exit 1
    python -c "import json,sys;d=json.loads(open('gpurun_out/ab_one.log').read().strip().splitlines()[-1]);print('${lib:-r06}', round(d['value']/1e9,2), d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['bucketing_stage']['ms_per_step'])"
  done
done
