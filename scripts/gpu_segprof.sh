#!/bin/bash
# Diagnostic: k_segments phase timing (a library built with -DOTM_SEG_PROF).
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r06_segprof}
mkdir -p $R/$O
cd $R
FAST="--no-check --no-cpu-baseline --host-steps 0 --json-calls 0 --stream-runs 0 --inflight 1"
timeout -k 10 400 python -u bench.py --config 4 --steps 3 --warmup 1 $FAST > $O/c4.out 2> $O/c4.err
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 $FAST > $O/c2.out 2> $O/c2.err
