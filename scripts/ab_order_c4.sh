#!/bin/bash
# Candidate work order A/B (OTM_ORDER_MASK=6: K2 in point order) on configs 2 and 4 -> gpurun_out/<tag>/
set -e
O=gpurun_out/${1:-order}
mkdir -p $O
FAST="--no-check --no-cpu-baseline --host-steps 0 --json-calls 0 --async-rounds 0 --single-requests 0"
for m in 7 6; do
  OTM_ORDER_MASK=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $FAST > $O/c2_m$m.json 2> $O/c2_m$m.err
  OTM_ORDER_MASK=$m timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 2 $FAST > $O/c4_m$m.json 2> $O/c4_m$m.err
done
