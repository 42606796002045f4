#!/bin/bash
# A/B of library builds in one call: variant "base" = reporter_amd/lib/
# libotmatch.so, any other name X = reporter_amd/lib/ab/libotmatch_X.so (via
# OTM_LIB).  Parity tests on every variant, then the device leg alternating
# the variants on config 2 (twice) and config 4 (once).
# Usage: bash scripts/gpu_abn.sh <tag> <variant>...
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/$1
shift
mkdir -p $R/$O
cd $R
lib() { if [ "$1" = base ]; then echo ""; else echo "$R/reporter_amd/lib/ab/libotmatch_$1.so"; fi; }
PT="tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_no_limits.py"
for v in "$@"; do
  OTM_LIB=$(lib $v) timeout -k 10 400 python -u -m pytest $PT -x -q --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1
done
FAST="--no-check --no-cpu-baseline --host-steps 0 --json-calls 0 --stream-runs 0"
for rep in 1 2; do
  for v in "$@"; do
    OTM_LIB=$(lib $v) timeout -k 10 200 python -u bench.py $FAST --steps 200 --warmup 10 > $O/bench_c2_${v}_$rep.json 2> $O/bench_c2_${v}_$rep.err
  done
done
for v in "$@"; do
  OTM_LIB=$(lib $v) timeout -k 10 400 python -u bench.py --config 4 --steps 10 --warmup 2 $FAST > $O/bench_c4_$v.json 2> $O/bench_c4_$v.err
done
