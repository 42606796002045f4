#!/bin/bash
# LDS bank-conflict A/B of library builds (PMC SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
# and a kernel trace per build, config 2, one batch in flight):
#   bash scripts/lds_ab.sh base noswz tudiag ...   -> gpurun_out/lds/<variant>/
set -e
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-check --host-steps 0 --json-calls 0 --traffic-json none --inflight 1"
for v in "$@"; do
  if [ "$v" = base ]; then L=$R/reporter_amd/lib/libotmatch.so; else L=$R/reporter_amd/lib/variants/$v/libotmatch.so; fi
  O=$R/gpurun_out/lds/$v
  mkdir -p $O
  OTM_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --output-format csv -d $O/pmc -o pmc -- $BENCH > $O/pmc.log 2>&1
  OTM_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- $BENCH > $O/kt.log 2>&1
done
