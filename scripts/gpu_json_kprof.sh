#!/bin/bash
# One-call JSON path (scripts/bench_json.py: otm_report_batch of 10k Java
# bodies, 7 calls) under a kernel + memory-copy trace: each JSON-path kernel's
# time with nothing else on the GPU, and the last call's timeline.
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_jkprof}
mkdir -p $R/$O
cd $R
(cd /tmp && export TMPDIR=/tmp && OTM_JSON_PROFILE=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats \
  --output-format csv -d $R/$O/trace -o run -- python3 $R/scripts/bench_json.py > $R/$O/run.json 2> $R/$O/run.err)
D=$(dirname $(find $R/$O/trace -name run_kernel_trace.csv | head -1))
python3 scripts/timeline.py $D 4 > $R/$O/timeline.txt
