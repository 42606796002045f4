#!/bin/bash
# Round 5: otm_report_batch split over the batch contexts -- the JSON/report
# GPU tests, then bench.py's JSON legs with the tree's library against
# reporter_amd/lib/variants/<B> (one batch per call), alternating, twice each.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_split}
B=${2:-nosplit}
mkdir -p $R/$O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_report.py tests/test_gpu_requests.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_json.log 2>&1
J="--steps 5 --warmup 2 --no-cpu-baseline --no-check --host-steps 0 --json-calls 5"
for i in 1 2; do
  OTM_JSON_PROFILE=1 timeout -k 10 300 python -u bench.py $J > $O/a_$i.json 2> $O/a_$i.err
  OTM_JSON_PROFILE=1 OTM_LIB=$R/reporter_amd/lib/variants/$B/libotmatch.so timeout -k 10 300 python -u bench.py $J > $O/b_$i.json 2> $O/b_$i.err
done
