#!/bin/bash
# Occupancy sensitivity of C3: extra LDS slack per document (MTR_SLACK) lowers the documents resident per CU;
# the kernel-trace pass of the default gives the launch mix.  usage: bash scripts/occ_sweep.sh <tag> [lib]
set -e
OUT=gpurun_out/occ_${1:-r04}
export MTR_LIB=${2:-libmtr.so}
mkdir -p $OUT
B="--steps 3 --warmup 1 --e2e-steps 0 --no-cpu-baseline"
for slack in 8 72 200; do
  MTR_SLACK=$slack timeout -k 10 200 python3 -u bench.py $B > $OUT/s$slack.json 2> $OUT/s$slack.err
done
echo done > $OUT/done
