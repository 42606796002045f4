#!/bin/bash
# Kernel + memory-copy traces of the host-inclusive leg, compact and SoA
# apart (4 batches in flight), and each leg alone over 5 rounds.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_host3}
mkdir -p $R/$O
cd $R
for leg in compact soa; do
  LEG=$leg ROUNDS=5 INFLIGHT=4 timeout -k 10 200 python -u scripts/host_leg.py > $O/alone_$leg.json 2> $O/alone_$leg.err
  (cd /tmp && export TMPDIR=/tmp && LEG=$leg ROUNDS=1 STEPS=20 INFLIGHT=4 timeout -k 10 300 rocprofv3 --kernel-trace \
    --memory-copy-trace --output-format csv -d $R/$O/trace_$leg -o run -- python3 $R/scripts/host_leg.py \
    > $R/$O/trace_$leg.log 2>&1)
done
