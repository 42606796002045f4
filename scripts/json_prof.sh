#!/bin/bash
# Kernel + copy trace of the JSON /report path (scripts/bench_json.py) -> gpurun_out/jprof/
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/jprof
cd /tmp && export TMPDIR=/tmp
OTM_GPU_JSON=${OTM_GPU_JSON:-1} timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
  -d $R/gpurun_out/jprof -o run -- python3 $R/scripts/bench_json.py > $R/gpurun_out/jprof/log.txt 2>&1
