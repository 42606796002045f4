set -e
mkdir -p gpurun_out/async
run() { name=$1; shift; env "$@" timeout -k 10 200 python -u scripts/bench_async.py > gpurun_out/async/$name.json 2> gpurun_out/async/$name.err; }
run w3t16 OTM_HOST_THREADS=16
run w3t12 OTM_HOST_THREADS=12
run w3t8 OTM_HOST_THREADS=8
run w2t12 OTM_HOST_THREADS=12 OTM_ASYNC_WORKERS=2
