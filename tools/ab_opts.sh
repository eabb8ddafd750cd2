#!/bin/bash
# A/B of handle options on one bench workload, on the GPU box: every option set runs ROUNDS times,
# interleaved, each its own bench.py process; one JSON line each into gpurun_out/ab_TAG_*.json.
#   tools/ab_opts.sh TAG ROUNDS "WORKLOAD ARGS" "OPTSET1" "OPTSET2" ...
# an option set is a space-separated list of NAME=VALUE (graindispatch.OPTIONS), "-" for the defaults;
#   e.g. tools/ab_opts.sh staged 2 "--workload cfg3 --steps 20 --warmup 5" "-" "l2_staged=0"
set -o pipefail
TAG=$1; ROUNDS=$2; ARGS=$3; shift 3
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out"
for r in $(seq 1 "$ROUNDS"); do
  i=0
  for SET in "$@"; do
    i=$((i+1))
    OPTS=()
    if [ "$SET" != "-" ]; then for kv in $SET; do OPTS+=(--opt "$kv"); done; fi
    OUT="$ROOT/gpurun_out/ab_${TAG}_${i}_${r}.json"
    timeout -k 10 300 python3 "$ROOT/bench.py" $ARGS --no-cpu-baseline --latency-batches 0 --no-secondary "${OPTS[@]}" \
        > "$OUT" 2> "$OUT.err" || { echo "set $i round $r failed"; tail -5 "$OUT.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); st=(d.get('roofline') or {}).get('bucketing_stage') or {}; print(sys.argv[2], 'round', sys.argv[3], round(d['value']/1e9,3), 'G/s', d['ms_per_step'], 'ms/step, stage', st.get('ms_per_step'))" "$OUT" "[$SET]" "$r"
  done
done
