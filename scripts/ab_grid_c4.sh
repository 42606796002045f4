#!/bin/bash
# Candidate grid multiplier A/B (OTM_GRID_MULT; 0 = the engine's model) on
# config 4 (200 m radius) and config 2, and batches in flight -> gpurun_out/<tag>/
set -e
O=gpurun_out/${1:-gridab}
mkdir -p $O
FAST="--no-check --no-cpu-baseline --host-steps 0 --json-calls 0 --async-rounds 0 --single-requests 0"
for m in 0 3 4 8; do
  OTM_GRID_MULT=$m timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 2 $FAST > $O/c4_m$m.json 2> $O/c4_m$m.err
done
for m in 0 1 3; do
  OTM_GRID_MULT=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $FAST > $O/c2_m$m.json 2> $O/c2_m$m.err
done
for f in 2 4; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --inflight $f $FAST > $O/c2_inf$f.json 2> $O/c2_inf$f.err
  timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 2 --inflight $f $FAST > $O/c4_inf$f.json 2> $O/c4_inf$f.err
done
