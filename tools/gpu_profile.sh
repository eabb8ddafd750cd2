#!/bin/bash
# Kernel-trace statistics + PMC counter passes for one bench.py configuration, on the GPU box.
#   tools/gpu_profile.sh TAG [extra bench.py args]
# Writes gpurun_out/prof_TAG/{trace,pmc_*}/ (CSV) and the summaries
# gpurun_out/prof_TAG/kernel_stats.csv, gpurun_out/prof_TAG/pmc_summary.json.
# Each pass has its own time limit; the script stops at the first failure.
set -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
# --latency-batches 0: no cfg 5 / cfg 1 secondary lines (their small launches would mix into the
# cfg 2 kernels' statistics and counters)
BENCH=(python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --profile-steps 0 --latency-batches 0 "$@")
cd /tmp || exit 1
echo "[profile $TAG] kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- "${BENCH[@]}" \
    > "$OUT/trace.log" 2>&1 || { echo "trace failed rc=$?"; tail -20 "$OUT/trace.log"; exit 1; }
PASSES=(
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
  "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
  "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
  "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"
)
i=0
for P in "${PASSES[@]}"; do
  i=$((i+1))
  echo "[profile $TAG] pmc pass $i: $P"
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/pmc_$i" -o run -- "${BENCH[@]}" \
      > "$OUT/pmc_$i.log" 2>&1 || { echo "pmc pass $i failed rc=$?"; tail -20 "$OUT/pmc_$i.log"; exit 1; }
done
cd "$ROOT" || exit 1
python3 tools/pmc_summary.py "$OUT"/pmc_* --json "$OUT/pmc_summary.json" > "$OUT/pmc_summary.txt" || exit 1
STATS=$(find "$OUT/trace" -name '*kernel_stats.csv' | head -1)
[ -n "$STATS" ] && cp "$STATS" "$OUT/kernel_stats.csv"
echo "[profile $TAG] done"
