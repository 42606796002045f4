#!/bin/bash
# Round 5: batch-context and copy streams created with a full CU mask (each its
# own hardware queue; variant cus) against the runtime's queue pool (the tree):
# the JSON/report GPU tests of the variant, then the bench alternating.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_cus}
mkdir -p $R/$O
cd $R
V=$R/reporter_amd/lib/variants/cus/libotmatch.so
OTM_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_report.py tests/test_gpu_requests.py tests/test_gpu_group.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_cus.log 2>&1
J="--no-cpu-baseline --no-check --json-calls 5 --single-requests 0"
for i in 1 2; do
  timeout -k 10 400 python -u bench.py $J > $O/a_$i.json 2> $O/a_$i.err
  OTM_LIB=$V timeout -k 10 400 python -u bench.py $J > $O/b_$i.json 2> $O/b_$i.err
done
