#!/bin/bash
# Round 5: configs 4 and 3 with the final bench defaults.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05c34}
mkdir -p $R/$O
cd $R
timeout -k 10 500 python -u bench.py --config 4 --steps 10 --warmup 2 --traffic-json profiles/r05_final/pmc_traffic_r05fin_c4.json > $O/bench_c4.json 2> $O/bench_c4.err
timeout -k 10 600 python -u bench.py --config 3 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err
