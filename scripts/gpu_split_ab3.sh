#!/bin/bash
# Round 5: the split's first-chunk share -- bench.py's JSON legs with the
# variants s40 / s50 / s60 (two chunks) and t50 (three), alternating.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_split3}
mkdir -p $R/$O
cd $R
J="--steps 5 --warmup 2 --no-cpu-baseline --no-check --host-steps 0 --json-calls 8 --async-rounds 0 --single-requests 0"
V=$R/reporter_amd/lib/variants
for i in 1 2; do
  for v in s40 s50 s60 t50; do
    OTM_LIB=$V/$v/libotmatch.so timeout -k 10 300 python -u bench.py $J > $O/${v}_$i.json 2> $O/${v}_$i.err
  done
done
