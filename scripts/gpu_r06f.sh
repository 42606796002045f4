#!/bin/bash
# Round 6: every GPU test (resume-at-the-grown-tier among them), kernel times
# on configs 2 and 4, and the redo-cost measurement (scripts/redo_cost.py).
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r06f}
mkdir -p $R/$O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
FAST="--no-check --no-cpu-baseline --host-steps 0 --json-calls 0 --stream-runs 0"
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py $FAST --steps 200 --warmup 10 > $O/bench_c2_$rep.json 2> $O/bench_c2_$rep.err
done
timeout -k 10 400 python -u bench.py --config 4 --steps 10 --warmup 2 $FAST > $O/bench_c4.json 2> $O/bench_c4.err
timeout -k 10 400 python -u scripts/redo_cost.py > $O/redo_cost.json 2> $O/redo_cost.err
