#!/bin/bash
# Round 5: the request reader's word-mask form (parity + one-call JSON kernel
# profile) and config 3's shard under forced index budgets (40 % tables; a
# budget that cuts the radius), each step under its own time limit.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05c}
mkdir -p $R/$O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_requests.py tests/test_gpu_report.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_json.log 2>&1
bash scripts/gpu_json_kprof.sh ${1:-r05c}/jk
FAST="--no-cpu-baseline --no-check --host-steps 0 --json-calls 0"
for mb in 75000 40000; do
  OTM_INDEX_BUDGET_MB=$mb timeout -k 10 500 python -u bench.py --config 3 --steps 5 --warmup 2 $FAST > $O/bench_c3_budget_$mb.json 2> $O/bench_c3_budget_$mb.err
done
