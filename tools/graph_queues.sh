#!/bin/bash
# hipGraph replay vs eager under HIP runtime graph settings (GPU box): tools/graph_queues.py per setting
set -u
mkdir -p gpurun_out
for q in - 1 2 4; do
  for pc in - 0; do
    E=()
    [ "$q" != - ] && E+=(DEBUG_HIP_FORCE_GRAPH_QUEUES=$q)
    [ "$pc" != - ] && E+=(DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc)
    env "${E[@]}" timeout -k 10 120 python tools/graph_queues.py 8 20 >> gpurun_out/graph_queues.log 2>&1 || exit 1
  done
done
DSR_STREAMS=1 timeout -k 10 120 python tools/graph_queues.py 8 20 >> gpurun_out/graph_queues.log 2>&1 || exit 1
cat gpurun_out/graph_queues.log
