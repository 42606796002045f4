#!/bin/bash
# Route-index A/B on config 2 (radius via --index-radius, load factor via
# variant builds): bench lines with the oracle check, one per setting.
#   bash scripts/ab_index.sh
set -e
mkdir -p gpurun_out/abi
run() {
  name=$1; lib=$2; shift 2
  OTM_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --host-steps 0 --json-calls 0 "$@" \
    > gpurun_out/abi/$name.json 2> gpurun_out/abi/$name.err
}
B=reporter_amd/lib/libotmatch.so
run base $B
run r900 $B --index-radius 900
run r700 $B --index-radius 700
run r500 $B --index-radius 500
run load33 reporter_amd/lib/variants/load33/libotmatch.so
run load50 reporter_amd/lib/variants/load50/libotmatch.so
run load50_r700 reporter_amd/lib/variants/load50/libotmatch.so --index-radius 700
