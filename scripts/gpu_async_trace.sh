#!/bin/bash
# The async JSON pipeline under a kernel + memory-copy trace (where a stalled
# run's time goes), and K5's time against the batch's trace count.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_atrace}
mkdir -p $R/$O
cd $R
(cd /tmp && export TMPDIR=/tmp && OTM_JSON_PROFILE=1 ARENA=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace \
  --output-format csv -d $R/$O/trace -o run -- python3 $R/scripts/bench_async.py > $R/$O/trace.json 2> $R/$O/trace.err)
FAST="--no-cpu-baseline --no-check --host-steps 0 --json-calls 0"
for v in 6000 8000 10000 12000 16000; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --vehicles $v $FAST > $O/vit_$v.json 2> $O/vit_$v.err
done
