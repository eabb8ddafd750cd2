# rocprofv3 kernel-trace statistics of the cfg 3 and cfg 4 bench lines (one GPU).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp || exit 1
for w in cfg3 cfg4; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_r03_$w -o run -- \
      python3 $ROOT/bench.py --workload $w --no-cpu-baseline --no-secondary --latency-batches 0 --profile-steps 0 --steps 10 --warmup 3 \
      > $ROOT/gpurun_out/prof_r03_$w.log 2>&1 || { tail -20 $ROOT/gpurun_out/prof_r03_$w.log; exit 1; }
done
