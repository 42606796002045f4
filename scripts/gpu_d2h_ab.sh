#!/bin/bash
# Host leg: result copies on the batch stream vs their own stream (OTM_D2H_STREAM=1),
# compact and SoA, 5 rounds each, 4 in flight; then a trace of the variant.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_d2h}
mkdir -p $R/$O
cd $R
for rep in 1 2; do
  for v in 0 1; do
    OTM_D2H_STREAM=$v ROUNDS=4 INFLIGHT=4 timeout -k 10 200 python -u scripts/host_leg.py > $O/d2h${v}_$rep.json 2> $O/d2h${v}_$rep.err
  done
done
(cd /tmp && export TMPDIR=/tmp && OTM_D2H_STREAM=1 LEG=compact ROUNDS=1 STEPS=20 INFLIGHT=4 timeout -k 10 300 rocprofv3 \
  --kernel-trace --memory-copy-trace --output-format csv -d $R/$O/trace -o run -- python3 $R/scripts/host_leg.py \
  > $R/$O/trace.log 2>&1)
# the async pipeline with per-batch phase lines (lock, push, read, match, write)
for rep in 1 2 3; do
  OTM_JSON_PROFILE=1 ARENA=1 timeout -k 10 200 python -u scripts/bench_async.py > $O/async_$rep.json 2> $O/async_$rep.err
done
