#!/bin/bash
# bench.py (config 2, with its JSON legs) under GPU_MAX_HW_QUEUES 4 (the
# runtime's default), 8 and 16 -> gpurun_out/<tag>/
set -e
O=gpurun_out/${1:-hwqb}
mkdir -p $O
for q in 4 16 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-check \
    > $O/q$q.json 2> $O/q$q.err
done
