#!/bin/bash
# Round 5: the round-end bench line with the final defaults (the PMC traffic
# of the final profile), the GPU tests and smoke(), each under its own limit.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05fb}
mkdir -p $R/$O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 400 python -u bench.py --traffic-json profiles/r05_final/pmc_traffic_r05fin.json > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
