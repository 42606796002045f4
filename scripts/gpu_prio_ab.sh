#!/bin/bash
# Round 5: the split call's copy stream from the runtime's high-priority queue
# pool (variant prio) against the pooled normal-priority one (the tree), the
# bench's default setup (four device contexts on own queues), JSON legs with
# phase lines, alternating.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_prio}
mkdir -p $R/$O
cd $R
J="--steps 20 --warmup 3 --no-cpu-baseline --no-check --json-calls 6 --single-requests 0"
V=$R/reporter_amd/lib/variants/prio/libotmatch.so
for i in 1 2; do
  OTM_JSON_PROFILE=1 timeout -k 10 300 python -u bench.py $J > $O/a_$i.json 2> $O/a_$i.err
  OTM_JSON_PROFILE=1 OTM_LIB=$V timeout -k 10 300 python -u bench.py $J > $O/b_$i.json 2> $O/b_$i.err
done
