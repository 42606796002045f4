#!/bin/bash
# PMC passes over a short bench run (one counter group per rocprofv3 run, as
# MI355X_MICROARCH.md's rocprofv3 section prescribes), then a JSON summary.
# HBM bytes come from the size-weighted DRAM request counters (32-byte units:
# a 64-byte request counts 2, a 128-byte one 4), so no FETCH_SIZE correction
# factor is needed; FETCH_SIZE / WRITE_SIZE and the request-size mix are kept
# beside them for comparison.
# Usage (on the GPU box, from the repo root): bash scripts/pmc.sh <out_dir> [tag]
set -e
R=$(pwd)
OUT=$R/${1:-gpurun_out/pmc}
TAG=${2:-latest}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-check --host-steps 0 --json-calls 0 --stream-runs 0 --traffic-json none --inflight 1 ${PMC_BENCH_ARGS:-}"
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- $BENCH > $OUT/$name.log 2>&1
}
pass dram TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum TCC_EA0_WRREQ_ATOMIC_DRAM_32B_sum
pass req TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass tcc TCC_HIT_sum TCC_MISS_sum
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
pass lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
cd $R
python3 scripts/pmc_summary.py $OUT $TAG ${PMC_STATS_CSV:-} > $OUT/pmc_traffic_$TAG.json
