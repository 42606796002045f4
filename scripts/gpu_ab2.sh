#!/bin/bash
# A/B of two library builds in one call: A = reporter_amd/lib/libotmatch.so,
# B = reporter_amd/lib/ab/libotmatch_B.so (OTM_LIB).  Parity tests on both,
# then the device leg alternating A, B on config 2 (twice) and config 4.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r06_ab2}
mkdir -p $R/$O
cd $R
B=$R/reporter_amd/lib/ab/libotmatch_B.so
PT="tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_no_limits.py"
timeout -k 10 400 python -u -m pytest $PT -x -q --timeout 300 --timeout-method thread > $O/pytest_A.log 2>&1
OTM_LIB=$B timeout -k 10 400 python -u -m pytest $PT -x -q --timeout 300 --timeout-method thread > $O/pytest_B.log 2>&1
FAST="--no-check --no-cpu-baseline --host-steps 0 --json-calls 0 --stream-runs 0"
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py $FAST --steps 200 --warmup 10 > $O/bench_c2_A$rep.json 2> $O/bench_c2_A$rep.err
  OTM_LIB=$B timeout -k 10 200 python -u bench.py $FAST --steps 200 --warmup 10 > $O/bench_c2_B$rep.json 2> $O/bench_c2_B$rep.err
done
timeout -k 10 400 python -u bench.py --config 4 --steps 10 --warmup 2 $FAST > $O/bench_c4_A.json 2> $O/bench_c4_A.err
OTM_LIB=$B timeout -k 10 400 python -u bench.py --config 4 --steps 10 --warmup 2 $FAST > $O/bench_c4_B.json 2> $O/bench_c4_B.err
