#!/bin/bash
# GPU tests (all, or the files given in OTM_TEST_FILES) then the default bench
# line, outputs under gpurun_out/quick/.  Any failing step ends the script.
set -e
mkdir -p gpurun_out/quick
timeout -k 10 600 python -u -m pytest ${OTM_TEST_FILES:-tests} -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/quick/pytest_gpu.log 2>&1
if [ "${OTM_BENCH:-1}" = "1" ]; then
  OTM_JSON_PROFILE=${OTM_JSON_PROFILE:-0} timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 ${OTM_BENCH_ARGS:-} \
    > gpurun_out/quick/bench.json 2> gpurun_out/quick/bench.err
fi
