#!/bin/bash
# Finer grid multiplier A/B on config 4 and a repeat of its in-flight depths -> gpurun_out/<tag>/
set -e
O=gpurun_out/${1:-gridab}
mkdir -p $O
FAST="--no-check --no-cpu-baseline --host-steps 0 --json-calls 0 --async-rounds 0 --single-requests 0"
for m in 6 8 10 12 16; do
  OTM_GRID_MULT=$m timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 2 $FAST > $O/c4_m$m.json 2> $O/c4_m$m.err
done
for f in 2 3; do
  OTM_GRID_MULT=8 timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 2 --inflight $f $FAST > $O/c4_m8_inf$f.json 2> $O/c4_m8_inf$f.err
done
