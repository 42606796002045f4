#!/bin/bash
# The async /report pipeline's phases (OTM_JSON_PROFILE=1: per-batch stage /
# gpu / copy-out lines and per-worker batch spans) and its kernel + copy trace
# -> gpurun_out/aprof/
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/aprof
OTM_JSON_PROFILE=1 timeout -k 10 200 python -u scripts/bench_async.py > gpurun_out/aprof/run.json 2> gpurun_out/aprof/run.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
  -d $R/gpurun_out/aprof/trace -o run -- python3 $R/scripts/bench_async.py > $R/gpurun_out/aprof/trace.log 2>&1
