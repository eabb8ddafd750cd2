# Round-4 validation on the GPU box: full GPU suite, the default bench line (driver style), the
# cfg 2 kernel-trace + PMC profile, and the cfg 3 / cfg 4 lines.   bash tools/run_r04.sh TAG
set -o pipefail
TAG=$1
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 2
timeout -k 10 300 python bench.py --workload cfg3 --steps 20 --warmup 5 --no-cpu-baseline --latency-batches 0 > gpurun_out/${TAG}_cfg3.json 2> gpurun_out/${TAG}_cfg3.err || exit 3
timeout -k 10 300 python bench.py --workload cfg4 --steps 5 --warmup 2 --no-cpu-baseline --latency-batches 0 > gpurun_out/${TAG}_cfg4.json 2> gpurun_out/${TAG}_cfg4.err || exit 4
echo "[run_r04 $TAG] done"
