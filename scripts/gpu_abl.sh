#!/bin/bash
# Ablation timing (builds that are wrong on purpose): device-leg kernel times
# of each variant, no parity tests.  Usage: bash scripts/gpu_abl.sh <tag> <variant>...
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/$1
shift
mkdir -p $R/$O
cd $R
lib() { if [ "$1" = base ]; then echo ""; else echo "$R/reporter_amd/lib/ab/libotmatch_$1.so"; fi; }
FAST="--no-check --no-cpu-baseline --host-steps 0 --json-calls 0 --stream-runs 0 --traffic-json none"
for v in "$@"; do
  OTM_LIB=$(lib $v) timeout -k 10 200 python -u bench.py $FAST --steps 50 --warmup 5 > $O/bench_c2_$v.json 2> $O/bench_c2_$v.err
  OTM_LIB=$(lib $v) timeout -k 10 400 python -u bench.py --config 4 --steps 5 --warmup 2 $FAST > $O/bench_c4_$v.json 2> $O/bench_c4_$v.err
done
