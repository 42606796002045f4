#!/bin/bash
# Batches in flight A/B on the device leg (config 2), two runs each
set -e
mkdir -p gpurun_out/abif
for n in 2 3 4 5; do
  for r in 1 2; do
    timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --inflight $n --no-cpu-baseline --no-check --host-steps 0 --json-calls 0 \
      > gpurun_out/abif/if$n.$r.json 2> gpurun_out/abif/if$n.$r.err
  done
done
