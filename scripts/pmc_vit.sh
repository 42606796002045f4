#!/bin/bash
# Viterbi A/B under PMC: kernel trace + SQ counter passes of a short config-2
# bench with OTM_VIT_FORM in PMC_FORMS (default "64 8") (GPU box, repo root): bash scripts/pmc_vit.sh <tag>
set -e
R=$(pwd)
TAG=${1:-vitpmc}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-check --host-steps 0 --json-calls 0 --async-rounds 0 --single-requests 0 --traffic-json none --inflight 1 ${PMC_BENCH_ARGS:-}"
for v in ${PMC_FORMS:-64 8}; do
  export OTM_VIT_FORM=$v
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt$v -o kt -- $BENCH > $OUT/kt$v.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $OUT/sq$v -o sq -- $BENCH > $OUT/sq$v.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_INST_LDS --output-format csv -d $OUT/sq2$v -o sq2 -- $BENCH > $OUT/sq2$v.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $OUT/lds$v -o lds -- $BENCH > $OUT/lds$v.log 2>&1
done
