#!/bin/bash
# GPU tests, then the config-2 and config-4 bench lines (outputs under
# gpurun_out/<tag>/).  Any failing step ends the script.
set -e
TAG=${1:-check}
O=gpurun_out/$TAG
mkdir -p $O
if [ "${OTM_TESTS:-1}" = "1" ]; then
  timeout -k 10 700 python -u -m pytest ${OTM_TEST_FILES:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1
fi
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 ${OTM_BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err
if [ "${OTM_C4:-1}" = "1" ]; then
  timeout -k 10 500 python -u bench.py --config 4 --steps 10 --warmup 2 ${OTM_BENCH_ARGS:-} > $O/bench_c4.json 2> $O/bench_c4.err
fi
