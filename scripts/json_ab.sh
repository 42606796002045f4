#!/bin/bash
# JSON /report path A/B: the GPU request reader against the host readers,
# phases per call (OTM_JSON_PROFILE=1) -> gpurun_out/json/
set -e
mkdir -p gpurun_out/json
for v in 1 0; do
  OTM_GPU_JSON=$v OTM_JSON_PROFILE=1 timeout -k 10 200 python -u scripts/bench_json.py > gpurun_out/json/gpu$v.json 2> gpurun_out/json/gpu$v.err
done
