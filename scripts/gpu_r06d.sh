#!/bin/bash
# Round 6: A/B of the route stage's work order (spatial order 7 vs natural
# point order 3 for K6), device leg, configs 2 and 4, alternated.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r06d}
mkdir -p $R/$O
cd $R
FAST="--no-check --no-cpu-baseline --host-steps 0 --json-calls 0 --stream-runs 0"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest_parity_default.log 2>&1
OTM_ORDER_MASK=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest_parity_mask3.log 2>&1
for rep in 1 2; do
  for m in 7 3; do
    OTM_ORDER_MASK=$m timeout -k 10 200 python -u bench.py $FAST --steps 200 --warmup 10 > $O/bench_c2_m${m}_$rep.json 2> $O/bench_c2_m${m}_$rep.err
  done
done
for m in 7 3; do
  OTM_ORDER_MASK=$m timeout -k 10 400 python -u bench.py --config 4 --steps 10 --warmup 2 $FAST > $O/bench_c4_m$m.json 2> $O/bench_c4_m$m.err
done
