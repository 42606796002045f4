#!/bin/bash
# Round 5: async pipeline depth and batch size (scripts/bench_async.py, arena
# bodies, 5 x 10k submissions), alternating, twice each.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_asweep}
mkdir -p $R/$O
cd $R
for i in 1 2; do
  for cfg in "3 16384" "2 16384" "2 32768" "3 32768"; do
    set -- $cfg
    ARENA=1 OTM_ASYNC_WORKERS=$1 OTM_ASYNC_BATCH=$2 timeout -k 10 150 python -u scripts/bench_async.py > $O/w$1_b$2_$i.json 2> $O/w$1_b$2_$i.err
  done
done
