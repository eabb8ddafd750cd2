#!/bin/bash
# After tools/gpu_profile.sh r05c{2,3,4} on the GPU box: the per-kernel PMC files bench.py reads
# (profiles/pmc_cfg*_*.json), the kernel statistics and counter summaries, here.   tools/pmc_refresh_local.sh TAG
set -e
TAG=${1:-final}
for c in 2 3 4; do
  d=gpurun_out/prof_r05c$c
  n=0; [ $c = 2 ] && n=16777216; [ $c = 3 ] && n=67108864
  python3 tools/pmc_traffic.py $d/pmc_summary.json r05_cfg${c}_$TAG cfg$c $n $d/kernel_stats.csv > /dev/null
  cp $d/kernel_stats.csv profiles/r05_cfg${c}_kernel_stats_final.csv
  cp $d/pmc_summary.txt profiles/r05_cfg${c}_pmc_summary.txt
done
# setup kernels (index builds, registration) are not bench kernels
git status --short profiles | awk '$1 == "??" {print $2}' | grep -E 'k_(cx8_build|cx_build|cx_types|cx_project|ctr_fold|reg_|lane_order|ring_owner)' | xargs -r rm
