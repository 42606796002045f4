#!/bin/bash
# Round 5: the device leg on library streams with hardware queues of their own
# (--own-queue-streams) against torch's streams, alternating, config 2 and 4.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_ownq}
mkdir -p $R/$O
cd $R
F="--no-cpu-baseline --no-check --host-steps 0 --json-calls 0"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 $F --own-queue-streams > $O/a2_$i.json 2> $O/a2_$i.err
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 $F > $O/b2_$i.json 2> $O/b2_$i.err
done
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --config 4 --steps 10 --warmup 2 $F --own-queue-streams > $O/a4_$i.json 2> $O/a4_$i.err
  timeout -k 10 400 python -u bench.py --config 4 --steps 10 --warmup 2 $F > $O/b4_$i.json 2> $O/b4_$i.err
done
