#!/bin/bash
# Bench configs (default "2 3") under several env settings, with the oracle check:
#   bash scripts/ab_env_configs.sh "" "OTM_TRANS_SUB=8" ...   ("" = defaults)
set -e
mkdir -p gpurun_out/abe
i=0
for setting in "$@"; do
  for c in ${AB_CONFIGS:-2 3}; do
    S=20; [ $c != 2 ] && S=5
    env $setting timeout -k 10 300 python -u bench.py --config $c --steps $S --warmup 2 --no-cpu-baseline \
      > gpurun_out/abe/run$i.c$c.json 2> gpurun_out/abe/run$i.c$c.err
  done
  echo "$setting" > gpurun_out/abe/run$i.env
  i=$((i+1))
done
