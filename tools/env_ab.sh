#!/bin/bash
# A/B of two environment settings on one bench workload, interleaved.   tools/env_ab.sh TAG ROUNDS "BENCH ARGS" "VAR=A ..." "VAR=B ..."
set -o pipefail
TAG=$1; ROUNDS=$2; ARGS=$3; A=$4; B=$5
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out"
for r in $(seq 1 "$ROUNDS"); do
  for L in A B; do
    E=$A; [ $L = B ] && E=$B
    OUT="$ROOT/gpurun_out/abe_${TAG}_${L}_${r}.json"
    env $E timeout -k 10 300 python3 "$ROOT/bench.py" $ARGS --no-cpu-baseline --latency-batches 0 --no-secondary \
        --full-out "$OUT.full" > "$OUT" 2> "$OUT.err" || { echo "$L round $r failed"; tail -5 "$OUT.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=json.load(open(sys.argv[1]+'.full')).get('kernels',{}); print(sys.argv[2], 'round', sys.argv[3], round(d['value']/1e9,3), 'G/s', d['ms_per_step'], 'ms/step', {n: k[n]['ms_per_step'] for n in sorted(k, key=lambda n: -k[n]['ms_per_step'])[:5]})" "$OUT" "$L:$E" "$r"
  done
done
