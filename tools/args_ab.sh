#!/bin/bash
# A/B of two bench argument sets on one workload, interleaved.   tools/args_ab.sh TAG ROUNDS "COMMON ARGS" "A ARGS" "B ARGS"
set -o pipefail
TAG=$1; ROUNDS=$2; ARGS=$3; A=$4; B=$5
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out"
for r in $(seq 1 "$ROUNDS"); do
  for L in A B; do
    X=$A; [ $L = B ] && X=$B
    OUT="$ROOT/gpurun_out/aba_${TAG}_${L}_${r}.json"
    timeout -k 10 300 python3 "$ROOT/bench.py" $ARGS $X --no-cpu-baseline --latency-batches 0 --no-secondary --full-out "$OUT.full" \
        > "$OUT" 2> "$OUT.err" || { echo "$L round $r failed"; tail -5 "$OUT.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'round', sys.argv[3], round(d['value']/1e9,3), 'G/s', d['ms_per_step'], 'ms/step', d['gpu_event_ms_per_step'], 'ev ms/step')" "$OUT" "$L:$X" "$r"
  done
done
