#!/bin/bash
# A/B of the async pipeline's request copies: the tree's library (one shared
# copy stream, copy engine) against reporter_amd/lib/variants/<B> (round 5's
# copies on each context's batch stream), alternating, 3 runs each; then the
# JSON/async GPU tests of the tree's library.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_aab}
B=${2:-bstream}
mkdir -p $R/$O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_report.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_report.log 2>&1
for i in 1 2 3; do
  ARENA=1 OTM_JSON_PROFILE=1 timeout -k 10 120 python -u scripts/bench_async.py > $O/a_$i.json 2> $O/a_$i.err
  ARENA=1 OTM_JSON_PROFILE=1 OTM_LIB=$R/reporter_amd/lib/variants/$B/libotmatch.so timeout -k 10 120 python -u scripts/bench_async.py > $O/b_$i.json 2> $O/b_$i.err
done
FAST="--no-cpu-baseline --no-check --host-steps 0 --json-calls 0"
OTM_INDEX_BUDGET_MB=60000 timeout -k 10 500 python -u bench.py --config 3 --steps 5 --warmup 2 $FAST > $O/bench_c3_budget_60000.json 2> $O/bench_c3_budget_60000.err
