#!/bin/bash
# Launch-policy sweep at the 8-GPU strong-scaling share (12,500 documents per GPU) and at C3's 100,000:
# ops per launch x LDS slack (MTR_SLACK).  usage: bash scripts/launch_sweep.sh <tag> [lib]
set -e
TAG=${1:-r04}
export MTR_LIB=${2:-libmtr.so}
OUT=gpurun_out/sweep_$TAG
mkdir -p $OUT
B="--steps 3 --warmup 1 --e2e-steps 0 --no-cpu-baseline"
for docs in 12500; do
  for k in 48 128 512; do
    for slack in 8 48; do
      MTR_SLACK=$slack timeout -k 10 200 python3 -u bench.py $B --docs $docs --ops-per-launch $k > $OUT/d${docs}_k${k}_s${slack}.json 2> $OUT/d${docs}_k${k}_s${slack}.err
    done
  done
done
echo done > $OUT/done
