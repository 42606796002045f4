#!/bin/bash
# Secondary bench lines (configs 3 and 4) with config 4's kernel trace and
# PMC passes.  GPU box, repo root: bash scripts/gpu_configs.sh <tag>
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-latest}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u bench.py --config 3 --steps 5 --warmup 2 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c4 -o run -- python3 $R/bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline --no-check --inflight 1 > $R/gpurun_out/prof_c4.log 2>&1)
PMC_BENCH_ARGS="--config 4" PMC_STATS_CSV=$R/gpurun_out/prof_c4/run_kernel_stats.csv bash scripts/pmc.sh gpurun_out/pmc_c4 c4_$TAG
timeout -k 10 400 python -u bench.py --config 4 --steps 5 --warmup 2 --traffic-json gpurun_out/pmc_c4/pmc_traffic_c4_$TAG.json > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
