set -e
mkdir -p gpurun_out/async
run() { name=$1; shift; env "$@" timeout -k 10 200 python -u scripts/bench_async.py > gpurun_out/async/$name.json 2> gpurun_out/async/$name.err; }
run w1b8k OTM_ASYNC_WORKERS=1 OTM_ASYNC_BATCH=8192
run w2b8k OTM_ASYNC_WORKERS=2 OTM_ASYNC_BATCH=8192
run w2b10k OTM_ASYNC_WORKERS=2 OTM_ASYNC_BATCH=10000
run w3b10k OTM_ASYNC_WORKERS=3 OTM_ASYNC_BATCH=10000
run w2b5k OTM_ASYNC_WORKERS=2 OTM_ASYNC_BATCH=5000
OTM_JSON_PROFILE=1 OTM_ASYNC_WORKERS=2 OTM_ASYNC_BATCH=10000 timeout -k 10 200 python -u scripts/bench_async.py > gpurun_out/async/prof.json 2> gpurun_out/async/prof.err
