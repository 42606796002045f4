#!/bin/bash
# GPU tests, then the bench at 3 (default), 1 and 4 batches in flight.
# Run from the repo root via gpurun; outputs under gpurun_out/.
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench3.json 2> gpurun_out/bench3.err
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-check --inflight 1 > gpurun_out/bench1.json 2>> gpurun_out/bench3.err
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-check --inflight 4 > gpurun_out/bench4.json 2>> gpurun_out/bench3.err
