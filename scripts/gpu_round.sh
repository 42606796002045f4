#!/bin/bash
# One GPU round on the MI355X box (run from the repo root via gpurun):
# GPU parity tests, the bench line, a kernel-trace profile of the same bench
# command and the PMC passes.  Outputs under gpurun_out/.
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-latest}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-check > $R/gpurun_out/prof.log 2>&1)
# the same bench with one batch in flight: kernel averages without overlap
# (the bench's roofline times its kernels one batch at a time)
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof1 -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-check --inflight 1 > $R/gpurun_out/prof1.log 2>&1)
if [ "${OTM_PMC:-1}" = "1" ]; then PMC_STATS_CSV=$R/gpurun_out/prof1/run_kernel_stats.csv bash scripts/pmc.sh gpurun_out/pmc $TAG; fi
