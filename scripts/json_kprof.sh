#!/bin/bash
# Kernel-trace stats of the JSON paths (scripts/bench_async.py: async runs and
# the one-call leg, ROUNDS=2) -> gpurun_out/<tag>/
set -e
R=$(pwd)
O=$R/gpurun_out/${1:-jkprof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ROUNDS=2 OTM_JSON_PROFILE=1 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/kt -o kt -- python3 $R/scripts/bench_async.py > $O/run.json 2> $O/run.err
