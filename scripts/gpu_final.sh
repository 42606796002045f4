#!/bin/bash
# Round-end evidence on the MI355X box (from the repo root via gpurun), in two
# calls that each fit one gpurun limit:
#   PART=1: GPU parity tests, config-2 kernel-trace profile + PMC passes, the
#           config-2 bench line carrying that PMC traffic, smoke();
#   PART=2: the same for config 4, then the config-3 shard line.
# Outputs under gpurun_out/<tag>/.  Any failing step ends the script.
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-final}
O=gpurun_out/$TAG
mkdir -p $R/$O
cd $R
FAST="--no-cpu-baseline --no-check --host-steps 0 --json-calls 0 --stream-runs 0 --inflight 1"
if [ "${PART:-1}" = "1" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof1 -o run -- python3 $R/bench.py --steps 10 --warmup 3 $FAST > $R/$O/prof1.log 2>&1)
  PMC_STATS_CSV=$R/$O/prof1/run_kernel_stats.csv bash scripts/pmc.sh $O/pmc $TAG
  timeout -k 10 400 python -u bench.py --traffic-json $O/pmc/pmc_traffic_$TAG.json > $O/bench.json 2> $O/bench.err
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
else
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof1c4 -o run -- python3 $R/bench.py --config 4 --steps 5 --warmup 2 $FAST > $R/$O/prof1c4.log 2>&1)
  PMC_BENCH_ARGS="--config 4" PMC_STATS_CSV=$R/$O/prof1c4/run_kernel_stats.csv bash scripts/pmc.sh $O/pmc4 ${TAG}_c4
  timeout -k 10 500 python -u bench.py --config 4 --steps 10 --warmup 2 --traffic-json $O/pmc4/pmc_traffic_${TAG}_c4.json > $O/bench_c4.json 2> $O/bench_c4.err
  timeout -k 10 600 python -u bench.py --config 3 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err
fi
