#!/bin/bash
# Stall / issue PMC passes (address and data stalls in TA/TCP, L1->L2 read
# requests and their latency, instruction mix, wave levels) over a short
# bench run, one counter group per rocprofv3 run within the per-block limits
# (8 SQ, 4 TCP, 2 TA), then the per-kernel summary of scripts/pmc_summary.py.
# Usage (on the GPU box, from the repo root): bash scripts/pmc_stall.sh <out_dir> [tag]
set -e
R=$(pwd)
OUT=$R/${1:-gpurun_out/stall}
TAG=${2:-stall}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-check --host-steps 0 --traffic-json none --inflight 1 ${PMC_BENCH_ARGS:-}"
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- $BENCH > $OUT/$name.log 2>&1
}
pass ta TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum
pass ta2 TA_DATA_STALLED_BY_TC_CYCLES_sum TA_TA_BUSY_sum
pass tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum
pass sq2 SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES
pass sq3 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE
cd $R
python3 scripts/pmc_summary.py $OUT $TAG ${PMC_STATS_CSV:-} > $OUT/pmc_$TAG.json
