#!/bin/bash
# Bench (configs 2 and 4 by default, with the oracle check) over variant builds:
#   bash scripts/ab_variants.sh base circle hash3 ...   ("base" = reporter_amd/lib/libotmatch.so)
#   AB_CONFIGS="2 3 4" bash scripts/ab_variants.sh ...
set -e
mkdir -p gpurun_out/abv
for v in "$@"; do
  if [ "$v" = base ]; then L=reporter_amd/lib/libotmatch.so; else L=reporter_amd/lib/variants/$v/libotmatch.so; fi
  for c in ${AB_CONFIGS:-2 4}; do
    S=20; [ $c != 2 ] && S=5
    OTM_LIB=$L timeout -k 10 300 python -u bench.py --config $c --steps $S --warmup 2 --no-cpu-baseline ${AB_BENCH_FLAGS:-} \
      > gpurun_out/abv/$v.c$c.json 2> gpurun_out/abv/$v.c$c.err
  done
done
