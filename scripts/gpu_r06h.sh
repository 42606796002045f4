#!/bin/bash
# Round 6: parity tests + device-leg kernel times (configs 2 and 4) for a
# kernel change.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r06h}
mkdir -p $R/$O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_no_limits.py -x -q --timeout 300 --timeout-method thread > $O/pytest_parity.log 2>&1
FAST="--no-check --no-cpu-baseline --host-steps 0 --json-calls 0 --stream-runs 0"
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py $FAST --steps 200 --warmup 10 > $O/bench_c2_$rep.json 2> $O/bench_c2_$rep.err
done
timeout -k 10 400 python -u bench.py --config 4 --steps 10 --warmup 2 $FAST > $O/bench_c4.json 2> $O/bench_c4.err
