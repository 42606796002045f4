#!/bin/bash
# The JSON /report paths' A/B (scripts/bench_async.py: async points/s and the
# one-call figure) over the pipelined otm_report_batch's chunk count
# (OTM_PIPE_CHUNKS, 1 = one batch) and the async workers' ordered copies
# (OTM_ASYNC_ORDER) -> gpurun_out/<tag>/
set -e
O=gpurun_out/${1:-pipe}
mkdir -p $O
for v in "OTM_PIPE_CHUNKS=1 OTM_ASYNC_ORDER=0" "OTM_PIPE_CHUNKS=4 OTM_ASYNC_ORDER=1" "OTM_PIPE_CHUNKS=3 OTM_ASYNC_ORDER=1" \
         "OTM_PIPE_CHUNKS=6 OTM_ASYNC_ORDER=1 OTM_ASYNC_BATCH=5000" "OTM_PIPE_CHUNKS=2 OTM_ASYNC_ORDER=1 OTM_ASYNC_WORKERS=4"; do
  tag=$(echo $v | tr ' =' '__')
  timeout -k 10 200 env $v python -u scripts/bench_async.py > $O/async_$tag.json 2> $O/async_$tag.err
done
