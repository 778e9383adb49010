#!/bin/bash
# One-GPU prediction of the driver's 8-GPU strong-scaling curve: C3's 100,000 documents split over
# N = 1, 2, 4, 8 ranks leave 100k / N documents per GPU; each is run here on one MI355X.
# usage: bash scripts/strong_predict.sh <tag>
set -e
TAG=${1:-r03}
OUT=gpurun_out/strong_$TAG
mkdir -p $OUT
for n in 100000 50000 25000 12500; do
  timeout -k 10 300 python3 -u bench.py --docs $n --steps 3 --warmup 1 --e2e-steps 0 --no-cpu-baseline > $OUT/c3_$n.json 2> $OUT/c3_$n.err
done
