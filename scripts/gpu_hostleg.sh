#!/bin/bash
# GPU tests, the bench line, and the host-inclusive leg alone: compact vs SoA
# (alternating) at 3 and 4 batches in flight.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_host}
mkdir -p $R/$O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
timeout -k 10 200 python -u scripts/host_leg.py > $O/host_both.json 2> $O/host_both.err
INFLIGHT=4 timeout -k 10 200 python -u scripts/host_leg.py > $O/host_both_4.json 2> $O/host_both_4.err
