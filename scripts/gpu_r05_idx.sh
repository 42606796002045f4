#!/bin/bash
# Round 5: the KIN=4 candidate layout (parity, then config 2/4 A/B against
# the default build), configs 3 and 4 on the compact route index, and the
# async JSON pipeline with phase lines (request arena, then copied bodies).
set -e
O=gpurun_out/${1:-r05_idx}
mkdir -p $O
K4=reporter_amd/lib/variants/kin4/libotmatch.so
FAST="--no-cpu-baseline --no-check --host-steps 0 --json-calls 0"
OTM_LIB=$K4 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > $O/pytest_kin4.log 2>&1
for v in default kin4; do
  L=""; [ $v = kin4 ] && L=$K4
  OTM_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $FAST > $O/bench_c2_$v.json 2> $O/bench_c2_$v.err
  OTM_LIB=$L timeout -k 10 400 python -u bench.py --config 4 --steps 10 --warmup 2 $FAST > $O/bench_c4_$v.json 2> $O/bench_c4_$v.err
done
OTM_JSON_PROFILE=1 ARENA=1 timeout -k 10 200 python -u scripts/bench_async.py > $O/async_arena.json 2> $O/async_arena.err
OTM_JSON_PROFILE=1 ARENA=0 timeout -k 10 200 python -u scripts/bench_async.py > $O/async_copied.json 2> $O/async_copied.err
timeout -k 10 500 python -u bench.py --config 3 --steps 5 --warmup 2 $FAST > $O/bench_c3.json 2> $O/bench_c3.err
