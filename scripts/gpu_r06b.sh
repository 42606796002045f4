#!/bin/bash
# Round 6: every GPU test (the tier-growth failures, cap and a real
# out-of-HBM grow, among them), an A/B of the Viterbi form under the bench's
# four batches in flight (device leg only, alternated), and config-4 kernel
# times with the K7 edge records.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r06b}
mkdir -p $R/$O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
FAST="--no-check --no-cpu-baseline --host-steps 0 --json-calls 0 --stream-runs 0"
for rep in 1 2; do
  for f in 64 8 16; do
    OTM_VIT_FORM=$f timeout -k 10 200 python -u bench.py $FAST --steps 200 --warmup 10 > $O/bench_vit${f}_$rep.json 2> $O/bench_vit${f}_$rep.err
  done
done
timeout -k 10 400 python -u bench.py --config 4 --steps 10 --warmup 2 $FAST > $O/bench_c4.json 2> $O/bench_c4.err
