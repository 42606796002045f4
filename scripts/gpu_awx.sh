#!/bin/bash
# Round 5: the async workers on clones with hardware queues of their own (the
# tree) -- the JSON/report/group GPU tests, then two full bench lines.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_awx}
mkdir -p $R/$O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_report.py tests/test_gpu_requests.py tests/test_gpu_group.py tests/test_gpu_batcher.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
J="--no-cpu-baseline --no-check --json-calls 5 --single-requests 0"
for i in 1 2; do
  timeout -k 10 400 python -u bench.py $J > $O/a_$i.json 2> $O/a_$i.err
done
