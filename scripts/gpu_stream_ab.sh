#!/bin/bash
# Config-5 stream leg at 8, 16 and 12 host threads (alternating, twice).
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r06_sthr}
mkdir -p $R/$O
cd $R
FAST="--no-check --no-cpu-baseline --host-steps 0 --json-calls 0 --steps 5 --warmup 2 --stream-runs 3"
for rep in 1 2; do
  for t in 8 16 12; do
    timeout -k 10 200 python -u bench.py $FAST --stream-threads $t > $O/bench_t${t}_$rep.json 2> $O/bench_t${t}_$rep.err
  done
done
