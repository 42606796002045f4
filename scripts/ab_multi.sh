#!/bin/bash
# Short bench runs under several env settings: bash scripts/ab_multi.sh "A=1 B=2" "A=3" ...
set -e
mkdir -p gpurun_out/ab
i=0
for setting in "$@"; do
  env $setting timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-check > gpurun_out/ab/run$i.json 2> gpurun_out/ab/run$i.err
  echo "$setting" > gpurun_out/ab/run$i.env
  i=$((i+1))
done
