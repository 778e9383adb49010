#!/bin/bash
# LRU-heap floor A/B for the LDS replay classes (MTR_HEAP_DIV).  usage: bash scripts/r05_heapdiv.sh <tag> [divs]
set -e
OUT=gpurun_out/r05_heapdiv_$1
mkdir -p $OUT
for dv in ${2:-8 16 32}; do
  for cfg in C2 C3; do
    MTR_HEAP_DIV=$dv timeout -k 10 300 python3 -u bench.py --config $cfg --steps 2 --warmup 1 --e2e-steps 0 --no-cpu-baseline > $OUT/${cfg}_d$dv.json 2> $OUT/${cfg}_d$dv.err
  done
done
echo done > $OUT/done
