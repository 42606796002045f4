#!/bin/bash
# GPU tests, small-batch round trips and the config-5 stream (outputs under gpurun_out/).
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 200 python -u scripts/diag_small.py > gpurun_out/diag_small.log 2>&1
timeout -k 10 300 python -u scripts/bench_stream.py --threads 8 > gpurun_out/stream_t8.json 2> gpurun_out/stream.err
