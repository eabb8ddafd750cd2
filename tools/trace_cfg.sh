#!/bin/bash
# rocprofv3 kernel trace of one bench workload (steady steps), then the per-step timeline.
#   tools/trace_cfg.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/trace_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/t" -o run -- python3 "$ROOT/bench.py" \
    --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --profile-steps 0 --latency-batches 0 --full-out "$OUT/full.json" "$@" \
    > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
cd "$ROOT" || exit 1
KT=$(find "$OUT/t" -name '*kernel_trace.csv' | head -1)
python3 tools/trace_gaps.py "$KT" "${FIRST:-k_route_m}" 2 > "$OUT/gaps.txt"
