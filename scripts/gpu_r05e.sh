#!/bin/bash
# Round 5: every GPU test with the split JSON call and the shared async copy
# stream, then one full bench line.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05e}
mkdir -p $R/$O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
