#!/bin/bash
# Device leg at 3, 4, 5 and 6 batches in flight (alternating, twice).
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r06_infl}
mkdir -p $R/$O
cd $R
FAST="--no-check --no-cpu-baseline --host-steps 0 --json-calls 0 --stream-runs 0 --steps 200 --warmup 10"
for rep in 1 2; do
  for n in 4 5 6 3; do
    timeout -k 10 200 python -u bench.py $FAST --inflight $n > $O/bench_i${n}_$rep.json 2> $O/bench_i${n}_$rep.err
  done
done
