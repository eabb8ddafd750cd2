#!/bin/bash
# EA requests per k_fan_route dispatch at BASELINE cfg 4 (pinned variants: the 8-B index probe).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_cfg4_fan
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum --output-format csv \
    -d "$OUT/pmc" -o run -- python3 "$ROOT/bench.py" --workload cfg4 --tune pinned --steps 3 --warmup 1 \
    --profile-steps 0 --no-cpu-baseline --full-out "$OUT/full.json" > "$OUT/pmc.log" 2>&1 || exit 1
