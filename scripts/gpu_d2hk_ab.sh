#!/bin/bash
# The runtime's D2H copies (blit kernels on every CU) against the library's
# own copy kernel with W workgroups (OTM_D2H_KERNEL=W): async JSON pipeline and
# the host-inclusive leg.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_d2hk}
mkdir -p $R/$O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_report.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "arena or compact or json or async or pinned" > $O/pytest.log 2>&1
for rep in 1 2; do
  for wg in 0 16 32 64; do
    OTM_D2H_KERNEL=$wg ARENA=1 timeout -k 10 200 python -u scripts/bench_async.py > $O/async_w${wg}_$rep.json 2> $O/async_w${wg}_$rep.err
  done
  for wg in 0 32; do
    OTM_D2H_KERNEL=$wg LEG=compact ROUNDS=4 INFLIGHT=4 timeout -k 10 200 python -u scripts/host_leg.py > $O/host_w${wg}_$rep.json 2> $O/host_w${wg}_$rep.err
  done
done
