# Full GPU suite, the default bench line, then the kernel-trace + PMC profile of cfg 2 (tools/gpu_profile.sh).
#   bash tools/run_full.sh TAG
set -o pipefail
TAG=$1
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 2
bash tools/gpu_profile.sh $TAG || exit 3
