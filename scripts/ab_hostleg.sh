#!/bin/bash
# Host-inclusive leg A/B (bench --host-steps) over env settings / bench flags:
#   AB_SET=blit bash scripts/ab_hostleg.sh   -> gpurun_out/abh/<name>.json
set -e
mkdir -p gpurun_out/abh
run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-check --host-steps 40 \
    $BENCH_EXTRA > gpurun_out/abh/$name.json 2> gpurun_out/abh/$name.err
}
case "${AB_SET:-prio}" in
prio)
  python3 -c "import torch; print('stream priority range (least, greatest):', torch.cuda.Stream.priority_range())" > gpurun_out/abh/prio.txt
  run base OTM_NOP=1
  run prio_hi OTM_STREAM_PRIO=hi
  run prio_hi_0_lo OTM_STREAM_PRIO=hi,0,lo
  BENCH_EXTRA="--host-stagger-ms 0.45" run stagger OTM_NOP=1
  BENCH_EXTRA="--inflight 2" run prio_hi_2 OTM_STREAM_PRIO=hi
  BENCH_EXTRA="--inflight 4" run prio_hi_4 OTM_STREAM_PRIO=hi,0,0,lo
  run sdma1 HSA_ENABLE_SDMA=1
  ;;
blit)
  run base OTM_NOP=1
  run wg8 DEBUG_CLR_LIMIT_BLIT_WG=8
  run wg16 DEBUG_CLR_LIMIT_BLIT_WG=16
  run wg32 DEBUG_CLR_LIMIT_BLIT_WG=32
  run wg64 DEBUG_CLR_LIMIT_BLIT_WG=64
  BENCH_EXTRA="--inflight 4" run wg16_4 DEBUG_CLR_LIMIT_BLIT_WG=16
  run engine1 GPU_BLIT_ENGINE_TYPE=1
  ;;
nocu)
  run base OTM_NOP=1
  run nocu OTM_COPY_NOCU=1
  BENCH_EXTRA="--inflight 2" run nocu_2 OTM_COPY_NOCU=1
  BENCH_EXTRA="--inflight 4" run nocu_4 OTM_COPY_NOCU=1
  ;;
serial)
  run base OTM_NOP=1
  run serial OTM_COPY_SERIAL=1
  BENCH_EXTRA="--inflight 4" run serial_4 OTM_COPY_SERIAL=1
  BENCH_EXTRA="--inflight 2" run serial_2 OTM_COPY_SERIAL=1
  ;;
sync)
  run base OTM_NOP=1
  run sync OTM_COPY_SYNC=1
  run sync_serial OTM_COPY_SYNC=1 OTM_COPY_SERIAL=1
  ;;
kern)
  run base OTM_NOP=1
  run k32 OTM_COPY_KERNEL=32
  run k64 OTM_COPY_KERNEL=64
  run k16 OTM_COPY_KERNEL=16
  run k128 OTM_COPY_KERNEL=128
  ;;
esac
