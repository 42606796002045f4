#!/bin/bash
# Round 6: the config-5 GPU tests (oracle-anchored batcher, raw path) and the
# default bench line with its new stream_config5 block.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r06a}
mkdir -p $R/$O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_batcher.py -x -v --timeout 200 --timeout-method thread > $O/pytest_batcher.log 2>&1
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err
