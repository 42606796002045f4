#!/bin/bash
# Round 5: batches in flight on own-queue streams (2 / 3 / 4) against the
# default (3 on torch's streams), config 2, alternating.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_infq}
mkdir -p $R/$O
cd $R
F="--steps 40 --warmup 5 --no-cpu-baseline --no-check --host-steps 0 --json-calls 0"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $F --torch-streams --inflight 3 > $O/d3_$i.json 2> $O/d3_$i.err
  timeout -k 10 300 python -u bench.py $F --inflight 4 > $O/q4_$i.json 2> $O/q4_$i.err
  timeout -k 10 300 python -u bench.py $F --inflight 2 > $O/q2_$i.json 2> $O/q2_$i.err
  timeout -k 10 300 python -u bench.py $F --torch-streams --inflight 4 > $O/d4_$i.json 2> $O/d4_$i.err
done
