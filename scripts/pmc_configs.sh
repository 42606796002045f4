#!/bin/bash
# Kernel-trace stats and the PMC traffic passes (scripts/pmc.sh) of a short
# bench run on config 2 and config 4 -> gpurun_out/<tag>/c2, c4
set -e
R=$(pwd)
TAG=${1:-pmcc}
for c in ${PMC_CONFIGS:-2 4}; do
  O=$R/gpurun_out/$TAG/c$c
  mkdir -p $O
  A="--config $c --steps 2 --warmup 1"
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- \
     python3 $R/bench.py $A --no-cpu-baseline --no-check --host-steps 0 --json-calls 0 --traffic-json none --inflight 1 \
     > $O/kt.log 2>&1)
  PMC_BENCH_ARGS="$A" PMC_STATS_CSV=$O/kt/kt_kernel_stats.csv bash scripts/pmc.sh gpurun_out/$TAG/c$c r04_c$c
done
