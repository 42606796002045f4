#!/bin/bash
# Viterbi form A/B (OTM_VIT_FORM: 8 = 8 lanes per trace then 16 then the wave
# form, 16 = 16 lanes then the wave form, 64 = the wave form only) on
# configs 2 and 4 -> gpurun_out/<tag>/
set -e
O=gpurun_out/${1:-vform}
mkdir -p $O
FAST="--no-check --no-cpu-baseline --host-steps 0 --json-calls 0 --async-rounds 0 --single-requests 0"
for f in 64 8 16; do
  OTM_VIT_FORM=$f timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $FAST > $O/c2_f$f.json 2> $O/c2_f$f.err
  OTM_VIT_FORM=$f timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 2 $FAST > $O/c4_f$f.json 2> $O/c4_f$f.err
done
