#!/bin/bash
# Round 5: bench.py's JSON legs with the device legs' clones closed first
# (bench.py) against the previous bench (scripts/_bench_prev.py), alternating.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_qab}
mkdir -p $R/$O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_requests.py tests/test_gpu_report.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_json.log 2>&1
bash scripts/gpu_json_kprof.sh ${1:-r05_qab}/jk
J="--steps 5 --warmup 2 --no-cpu-baseline --no-check --json-calls 5 --single-requests 0"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $J > $O/a_$i.json 2> $O/a_$i.err
  PYTHONPATH=$R timeout -k 10 300 python -u scripts/_bench_prev.py $J > $O/b_$i.json 2> $O/b_$i.err
done
