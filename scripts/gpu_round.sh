#!/bin/bash
# One GPU round on the MI355X box (run from the repo root via gpurun):
# GPU parity tests, the bench line, a kernel-trace profile of the same bench
# command (one batch in flight, as the bench's kernel timers run) and the PMC
# passes.  Outputs under gpurun_out/.  Any failing step ends the script.
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-latest}
mkdir -p $R/gpurun_out
cd $R
if [ "${OTM_TESTS:-1}" = "1" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
fi
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof1 -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-check --host-steps 0 --json-calls 0 --inflight 1 > $R/gpurun_out/prof1.log 2>&1)
if [ "${OTM_PMC:-1}" = "1" ]; then PMC_STATS_CSV=$R/gpurun_out/prof1/run_kernel_stats.csv bash scripts/pmc.sh gpurun_out/pmc $TAG; fi
