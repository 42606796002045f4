#!/bin/bash
# GPU tests, the config-2 / config-4 bench lines, then the Viterbi A/B
# (OTM_VIT_SUB=0: the wave-per-trace form only) on the device legs.
# Outputs under gpurun_out/<tag>/.  Any failing step ends the script.
set -e
TAG=${1:-vit}
O=gpurun_out/$TAG
mkdir -p $O
if [ "${OTM_TESTS:-1}" = "1" ]; then
  timeout -k 10 700 python -u -m pytest ${OTM_TEST_FILES:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1
fi
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
timeout -k 10 500 python -u bench.py --config 4 --steps 10 --warmup 2 > $O/bench_c4.json 2> $O/bench_c4.err
FAST="--no-check --no-cpu-baseline --host-steps 0 --json-calls 0 --async-rounds 0 --single-requests 0"
for v in 0 1; do
  OTM_VIT_SUB=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $FAST > $O/ab_c2_sub$v.json 2> $O/ab_c2_sub$v.err
  OTM_VIT_SUB=$v timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 2 $FAST > $O/ab_c4_sub$v.json 2> $O/ab_c4_sub$v.err
done
