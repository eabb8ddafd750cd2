#!/bin/bash
# The N > 1 bench flow rehearsed on one GPU: torchrun, every rank on cuda:0, gloo with host-staged
# all-to-all (bench.py --rehearse-one-gpu).  tools/rehearse.sh N [bench args...]
set -o pipefail
N=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
    --master-port $((29600 + N)) "$ROOT/bench.py" --gpus "$N" --rehearse-one-gpu --no-cpu-baseline \
    --full-out "$ROOT/gpurun_out/rehearse_w${N}_full.json" "$@" \
    > "$ROOT/gpurun_out/rehearse_w${N}.json" 2> "$ROOT/gpurun_out/rehearse_w${N}.err"
