#!/bin/bash
# Round 5: the async pipeline's copy stream on a hardware queue of its own (the
# tree) against a pooled one (variant apool); the workers' batch streams on
# their own queues in both.  JSON/report GPU tests of the tree, then
# bench.py's JSON legs alternating.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_aorder}
mkdir -p $R/$O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_report.py tests/test_gpu_requests.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
J="--steps 5 --warmup 2 --no-cpu-baseline --no-check --host-steps 0 --json-calls 5 --single-requests 0"
V=$R/reporter_amd/lib/variants/apool/libotmatch.so
for i in 1 2; do
  OTM_JSON_PROFILE=1 timeout -k 10 300 python -u bench.py $J > $O/a_$i.json 2> $O/a_$i.err
  OTM_JSON_PROFILE=1 OTM_LIB=$V timeout -k 10 300 python -u bench.py $J > $O/b_$i.json 2> $O/b_$i.err
done
