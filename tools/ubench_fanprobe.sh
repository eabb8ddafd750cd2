#!/bin/bash
# tools/ubench_fanprobe on the GPU box: timings, then EA read requests per kernel (rocprofv3 --pmc).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/ubench_fanprobe
mkdir -p "$OUT"
export TMPDIR=/tmp
for shape in "25 43000000 0.3" "24 43000000 0.6" "21 16777216 0.5"; do
  echo "== shape $shape"
  timeout -k 10 120 "$ROOT/tools/ubench_fanprobe" $shape || exit 1
done > "$OUT/timings.txt" 2>&1
cd /tmp || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum --output-format csv \
    -d "$OUT/pmc" -o run -- "$ROOT/tools/ubench_fanprobe" 25 43000000 0.3 > "$OUT/pmc.log" 2>&1 || exit 1
