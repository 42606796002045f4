#!/bin/bash
# Round 5 route-index A/B: the compact index (default: 16-B slots with the
# predecessor inside, 2-slot buckets at 40 % load) against round 4's library
# (r04: 20-B slots at 20 %), single-slot first probes, and 30 % load.
set -e
O=gpurun_out/${1:-r05_abidx}
mkdir -p $O
FAST="--no-cpu-baseline --no-check --host-steps 0 --json-calls 0"
V="default r04 single load30 load30s"
lib() { [ $1 = default ] && echo "" || echo reporter_amd/lib/variants/$1/libotmatch.so; }
for rep in 1 2; do
  for v in $V; do
    OTM_LIB=$(lib $v) timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 $FAST > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err
  done
done
for v in $V; do
  OTM_LIB=$(lib $v) timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 2 $FAST > $O/c4_$v.json 2> $O/c4_$v.err
done
for v in default r04 load30; do
  OTM_LIB=$(lib $v) timeout -k 10 400 python -u bench.py --config 3 --steps 5 --warmup 2 $FAST > $O/c3_$v.json 2> $O/c3_$v.err
done
# (round 5 also ran the async pipeline here with its request copies on the
# batch stream or on a copy stream per context, bodies in a request arena or
# copied: no setting won every run, one stream per context kept)
