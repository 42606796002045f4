#!/bin/bash
# Round 5: the split call's second context on the engine's stream with the copy
# stream on its own hardware queue (the tree) against two pooled clones and a
# pooled copy stream (variant v2), bench.py's JSON legs with phase lines.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_sform}
mkdir -p $R/$O
cd $R
J="--steps 5 --warmup 2 --no-cpu-baseline --no-check --host-steps 0 --json-calls 8 --single-requests 0"
V=$R/reporter_amd/lib/variants/v2/libotmatch.so
for i in 1 2; do
  OTM_JSON_PROFILE=1 timeout -k 10 300 python -u bench.py $J > $O/a_$i.json 2> $O/a_$i.err
  OTM_JSON_PROFILE=1 OTM_LIB=$V timeout -k 10 300 python -u bench.py $J > $O/b_$i.json 2> $O/b_$i.err
done
