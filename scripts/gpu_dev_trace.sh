#!/bin/bash
# Round 5: a kernel trace of the device leg at three batches in flight (the
# bench's `value` configuration), for each kernel's share of the timeline.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_devtrace}
mkdir -p $R/$O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/trace -o run -- python3 $R/bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-check --host-steps 0 --json-calls 0 > $R/$O/bench.json 2> $R/$O/bench.err
