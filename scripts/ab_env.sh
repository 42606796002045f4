#!/bin/bash
# A/B of one env knob over short bench runs: bash scripts/ab_env.sh VAR v1 v2 ...
set -e
VAR=$1; shift
mkdir -p gpurun_out/ab
for v in "$@"; do
  env $VAR=$v timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-check > gpurun_out/ab/$VAR.$v.json 2> gpurun_out/ab/$VAR.$v.err
done
