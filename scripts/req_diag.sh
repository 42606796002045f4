#!/bin/bash
# k_req_scan diagnostics (OTM_REQ_DIAG: 0 full, 1 header only, 2 windows without point parsing)
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for m in 0 1 2; do
  mkdir -p $R/gpurun_out/rdiag/m$m
  OTM_REQ_DIAG=$m OTM_JSON_VEH=3000 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $R/gpurun_out/rdiag/m$m -o run -- python3 $R/scripts/bench_json.py > $R/gpurun_out/rdiag/m$m/log.txt 2>&1 || true
done
