#!/bin/bash
# Config-5 stream benches (scripts/bench_stream.py) on the GPU box; outputs under gpurun_out/.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_batcher.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_batcher.log 2>&1
timeout -k 10 300 python -u scripts/bench_stream.py --threads 1 --cpu-sample 0 > gpurun_out/stream_t1.json 2> gpurun_out/stream.err
timeout -k 10 300 python -u scripts/bench_stream.py --threads 8 > gpurun_out/stream_t8.json 2>> gpurun_out/stream.err
timeout -k 10 300 python -u scripts/bench_stream.py --threads 16 --cpu-sample 0 > gpurun_out/stream_t16.json 2>> gpurun_out/stream.err
timeout -k 10 300 python -u scripts/bench_stream.py --threads 8 --raw json --format-threads 16 --cpu-sample 0 > gpurun_out/stream_rawjson.json 2>> gpurun_out/stream.err
timeout -k 10 300 python -u scripts/bench_stream.py --threads 8 --vehicles 100000 --chunk 200000 --max-pending 1000000 --cpu-sample 0 > gpurun_out/stream_100k.json 2>> gpurun_out/stream.err
