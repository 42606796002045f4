#!/bin/bash
# One-call JSON path over its chunk count, with the runtime's default hardware
# queues and with 16 (GPU_MAX_HW_QUEUES; each batch context holds two or three
# streams) -> gpurun_out/<tag>/
set -e
O=gpurun_out/${1:-hwq}
mkdir -p $O
for q in 4 16; do
  for c in 1 2 4; do
    GPU_MAX_HW_QUEUES=$q OTM_PIPE_CHUNKS=$c OTM_JSON_PROFILE=1 timeout -k 10 200 python -u scripts/bench_async.py > $O/q${q}_c$c.json 2> $O/q${q}_c$c.err
  done
done
