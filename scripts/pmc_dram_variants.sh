#!/bin/bash
# One DRAM-counter pass per variant build on one config (A/B of HBM traffic):
#   PMC_CONFIG=4 bash scripts/pmc_dram_variants.sh base bucket ...
set -e
R=$(pwd)
O=$R/gpurun_out/pmcv
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = base ]; then L=$R/reporter_amd/lib/libotmatch.so; else L=$R/reporter_amd/lib/variants/$v/libotmatch.so; fi
  OTM_LIB=$L timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum TCC_HIT_sum TCC_MISS_sum \
    --output-format csv -d $O/$v -o $v -- python3 $R/bench.py --config ${PMC_CONFIG:-4} --steps 2 --warmup 1 --no-cpu-baseline \
    --no-check --host-steps 0 --json-calls 0 --traffic-json none --inflight 1 > $O/$v.log 2>&1
done
