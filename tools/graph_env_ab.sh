#!/bin/bash
# A/B of the runtime's graph knobs around tools/ubench_graph (built on the CPU side:
#   hipcc --offload-arch=gfx950 -O3 tools/ubench_graph.hip -o tools/ubench_graph).
# Usage (GPU box): bash tools/graph_env_ab.sh > gpurun_out/graph_env_ab.txt
set -e
# DEBUG_HIP_FORCE_GRAPH_QUEUES=0 dies with SIGFPE inside the runtime (ROCm 7.2), so it is not in the list
for cfg in "" "DEBUG_HIP_FORCE_GRAPH_QUEUES=1" \
           "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" \
           "DEBUG_HIP_GRAPH_BATCH_SIZE=1" "HIP_FORCE_DEV_KERNARG=1" "DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0"; do
    echo "== ${cfg:-default}"
    if [ -n "$cfg" ]; then export "$cfg"; fi
    timeout -k 10 60 ./tools/ubench_graph
    if [ -n "$cfg" ]; then unset "${cfg%%=*}"; fi
done
