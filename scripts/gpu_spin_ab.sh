#!/bin/bash
# Round 5: the JSON batches' host waits spinning (variant spin) against
# blocking (the tree), bench.py's JSON legs, alternating.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_spin}
mkdir -p $R/$O
cd $R
J="--steps 5 --warmup 2 --no-cpu-baseline --no-check --host-steps 0 --json-calls 8 --single-requests 0"
V=$R/reporter_amd/lib/variants/spin/libotmatch.so
for i in 1 2; do
  OTM_JSON_PROFILE=1 timeout -k 10 300 python -u bench.py $J > $O/a_$i.json 2> $O/a_$i.err
  OTM_JSON_PROFILE=1 OTM_LIB=$V timeout -k 10 300 python -u bench.py $J > $O/b_$i.json 2> $O/b_$i.err
done
