#!/bin/bash
# A/B of whole library builds on one box (ABAB order against drift):
#   bash scripts/ab_layout.sh base v2old     ("base" = reporter_amd/lib/libotmatch.so,
#                                              others reporter_amd/lib/variants/<name>/libotmatch.so)
# AB_CONFIGS (default "2 4"), AB_ROUNDS (default 2); outputs gpurun_out/abl/<variant>.c<config>.<round>.json
set -e
mkdir -p gpurun_out/abl
for r in $(seq 1 ${AB_ROUNDS:-2}); do
  for c in ${AB_CONFIGS:-2 4}; do
    for v in "$@"; do
      if [ "$v" = base ]; then L=reporter_amd/lib/libotmatch.so; else L=reporter_amd/lib/variants/$v/libotmatch.so; fi
      S=30; [ $c != 2 ] && S=8
      OTM_LIB=$L timeout -k 10 300 python -u bench.py --config $c --steps $S --warmup 3 --no-cpu-baseline \
        --json-calls 0 --host-steps 0 > gpurun_out/abl/$v.c$c.$r.json 2> gpurun_out/abl/$v.c$c.$r.err
    done
  done
done
