#!/bin/bash
# Independent document groups (MTR_GROUPS) at the strong-scaling shares of C3: 100,000 / N documents on one
# MI355X for N = 1, 2, 4, 8, each with 1, 2 and 4 groups.  usage: bash scripts/groups_sweep.sh <tag> [lib]
set -e
TAG=${1:-r04}
export MTR_LIB=${2:-libmtr.so}
OUT=gpurun_out/groups_$TAG
mkdir -p $OUT
B="--steps 3 --warmup 1 --e2e-steps 0 --no-cpu-baseline"
for docs in 12500 25000 50000 100000; do
  for g in 1 2 4; do
    MTR_GROUPS=$g timeout -k 10 200 python3 -u bench.py $B --docs $docs > $OUT/d${docs}_g${g}.json 2> $OUT/d${docs}_g${g}.err
  done
done
echo done > $OUT/done
