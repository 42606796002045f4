#!/bin/bash
# Fast bench lines (no oracle check, no host/JSON legs) on configs 2 and 4 under
# several env settings:  bash scripts/ab_env_fast.sh <tag> "" "OTM_TRANS_SUB=16" ...
set -e
O=gpurun_out/${1:-abef}
shift
mkdir -p $O
FAST="--no-check --no-cpu-baseline --host-steps 0 --json-calls 0 --async-rounds 0 --single-requests 0"
i=0
for setting in "$@"; do
  for c in ${AB_CONFIGS:-2 4}; do
    S=20; [ $c != 2 ] && S=10
    env $setting timeout -k 10 300 python -u bench.py --config $c --steps $S --warmup 2 $FAST > $O/run$i.c$c.json 2> $O/run$i.c$c.err
  done
  echo "$setting" > $O/run$i.env
  i=$((i+1))
done
