#!/bin/bash
# Round 5 check: every GPU test, the default bench line, configs 4 and 3, and
# config 4's PMC passes (Viterbi LDS conflicts, index traffic).
set -e
O=gpurun_out/${1:-r05b}
mkdir -p $O
FAST="--no-cpu-baseline --no-check --host-steps 0 --json-calls 0"
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -v --timeout 300 --timeout-method thread -k index_budget > $O/pytest_budget.log 2>&1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 2 $FAST > $O/bench_c4.json 2> $O/bench_c4.err
timeout -k 10 400 python -u bench.py --config 3 --steps 5 --warmup 2 $FAST > $O/bench_c3.json 2> $O/bench_c3.err
PMC_BENCH_ARGS="--config 4" bash scripts/pmc.sh $O/pmc4 r05b_c4
