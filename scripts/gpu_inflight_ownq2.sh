#!/bin/bash
# Round 5: 4 / 5 / 6 batches in flight on own-queue streams against the
# default (3 on torch's streams), config 2, alternating.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_infq2}
mkdir -p $R/$O
cd $R
F="--steps 60 --warmup 5 --no-cpu-baseline --no-check --host-steps 0 --json-calls 0"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $F --torch-streams --inflight 3 > $O/d3_$i.json 2> $O/d3_$i.err
  for n in 4 5 6; do
    timeout -k 10 300 python -u bench.py $F --inflight $n > $O/q${n}_$i.json 2> $O/q${n}_$i.err
  done
done
