#!/bin/bash
# bench.py's JSON legs with the per-batch phase lines (OTM_JSON_PROFILE=1)
# -> gpurun_out/bprof/ (the async leg's runs as the bench sees them)
set -e
mkdir -p gpurun_out/bprof
OTM_JSON_PROFILE=1 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-check ${OTM_BENCH_ARGS:-} \
  > gpurun_out/bprof/bench${OTM_TAG:-}.json 2> gpurun_out/bprof/bench${OTM_TAG:-}.err
