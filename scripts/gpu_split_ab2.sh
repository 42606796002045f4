#!/bin/bash
# Round 5: otm_report_batch in two chunks (first 25 % of the bytes) against
# the 40 % variant and one batch per call (nosplit), bench.py's JSON legs,
# alternating; the split GPU test first.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_split2}
mkdir -p $R/$O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_report.py -m gpu -x -v --timeout 300 --timeout-method thread -k "split or arena" > $O/pytest_split.log 2>&1
J="--steps 5 --warmup 2 --no-cpu-baseline --no-check --host-steps 0 --json-calls 8 --async-rounds 0 --single-requests 0"
V=$R/reporter_amd/lib/variants
for i in 1 2; do
  OTM_JSON_PROFILE=1 timeout -k 10 300 python -u bench.py $J > $O/a_$i.json 2> $O/a_$i.err
  OTM_JSON_PROFILE=1 OTM_LIB=$V/nosplit/libotmatch.so timeout -k 10 300 python -u bench.py $J > $O/b_$i.json 2> $O/b_$i.err
  OTM_JSON_PROFILE=1 OTM_LIB=$V/s40/libotmatch.so timeout -k 10 300 python -u bench.py $J > $O/c_$i.json 2> $O/c_$i.err
done
