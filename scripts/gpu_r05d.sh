#!/bin/bash
# Round 5: the response copy kernel's LDS form -- JSON/report GPU tests, the
# one-call JSON kernel profile, and three async runs (arena).
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05d}
mkdir -p $R/$O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_requests.py tests/test_gpu_report.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_json.log 2>&1
bash scripts/gpu_json_kprof.sh ${1:-r05d}/jk
for i in 1 2 3; do
  ARENA=1 OTM_JSON_PROFILE=1 timeout -k 10 120 python -u scripts/bench_async.py > $O/a_$i.json 2> $O/a_$i.err
done
