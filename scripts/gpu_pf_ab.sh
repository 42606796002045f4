#!/bin/bash
# Round 5: K4's prefetching form (the next step's column record and candidate
# records loaded under this step's probes) -- parity tests, then configs 2
# and 4 against the variant without it (nopf), alternating.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_pf}
mkdir -p $R/$O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_no_limits.py tests/test_turn_route.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
F="--no-cpu-baseline --no-check --host-steps 0 --json-calls 0"
V=$R/reporter_amd/lib/variants/nopf/libotmatch.so
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 $F > $O/a2_$i.json 2> $O/a2_$i.err
  OTM_LIB=$V timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 $F > $O/b2_$i.json 2> $O/b2_$i.err
done
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --config 4 --steps 8 --warmup 2 $F > $O/a4_$i.json 2> $O/a4_$i.err
  OTM_LIB=$V timeout -k 10 400 python -u bench.py --config 4 --steps 8 --warmup 2 $F > $O/b4_$i.json 2> $O/b4_$i.err
done
