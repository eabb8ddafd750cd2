# L2 / SQ counters of the owner probe with and without the region mapping (tools/ab_region_serial.py)
#   bash tools/pmc_region.sh "COUNTERS" TAG
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
CTRS=${1:-"TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"}
TAG=${2:-l2}
cd /tmp || exit 1
for b in 0 1; do
  D="$ROOT/gpurun_out/pmc_region_${TAG}_$b"
  GD_REGION_PROBE=$b timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv \
      -d "$D" -o run -- python3 "$ROOT/tools/ab_region_serial.py" > "$D.log" 2>&1 || { echo "pmc $b failed"; tail -20 "$D.log"; exit 1; }
  echo "GD_REGION_PROBE=$b"; python3 "$ROOT/tools/pmc_summary.py" "$D" --kernel route || exit 1
done
