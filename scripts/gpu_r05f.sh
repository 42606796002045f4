#!/bin/bash
# Round 5: py_repr's 64-bit digit loop in the response writer -- the JSON /
# report GPU tests, the one-call JSON kernel profile, one bench line.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05f}
mkdir -p $R/$O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_requests.py tests/test_gpu_report.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_json.log 2>&1
bash scripts/gpu_json_kprof.sh ${1:-r05f}/jk
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-check > $O/bench.json 2> $O/bench.err
