#!/bin/bash
# Global search tier at index radii that leave transitions to the online tiers (config 2)
set -e
mkdir -p gpurun_out/abbig
run() {
  name=$1; shift
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --host-steps 0 --json-calls 0 "$@" \
    > gpurun_out/abbig/$name.json 2> gpurun_out/abbig/$name.err
}
run ${1:-cur}_r700 --index-radius 700
run ${1:-cur}_r0 --index-radius 0
