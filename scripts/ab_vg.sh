#!/bin/bash
# Grouped-Viterbi build A/B (scripts/build_variant.sh variants) on config 4 -> gpurun_out/<tag>/
set -e
O=gpurun_out/${1:-vgab}
mkdir -p $O
FAST="--no-check --no-cpu-baseline --host-steps 0 --json-calls 0 --async-rounds 0 --single-requests 0"
for v in base "$@"; do
  [ "$v" = "$1" ] && continue
  if [ "$v" = base ]; then L=reporter_amd/lib/libotmatch.so; else L=reporter_amd/lib/variants/$v/libotmatch.so; fi
  OTM_LIB=$L timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 2 $FAST > $O/$v.c4.json 2> $O/$v.c4.err
done
