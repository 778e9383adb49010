#!/bin/bash
# Long launches at the 8-GPU share of C3 (12,500 documents): ops per launch K, slack leaves S per document
# (MTR_SLACK), one size class (MTR_CLASS_LEAVES=1024) or the default 64-leaf classes, 1 or 2 groups.
# usage: bash scripts/launch_sweep.sh <tag>
set -e
TAG=${1:-r04}
OUT=gpurun_out/launch_$TAG
mkdir -p $OUT
B="--steps 3 --warmup 1 --e2e-steps 0 --no-cpu-baseline"
run() {  # name docs K env...
  local name=$1 docs=$2 k=$3; shift 3
  env "$@" timeout -k 10 200 python3 -u bench.py $B --docs $docs --ops-per-launch $k > $OUT/$name.json 2> $OUT/$name.err
}
run base_d12500 12500 48
for s in 64 192 448; do
  run k1000_s${s}_c1024_d12500 12500 1000 MTR_SLACK=$s MTR_CLASS_LEAVES=1024
  run k1000_s${s}_c64_d12500 12500 1000 MTR_SLACK=$s
done
run k250_s96_c1024_d12500 12500 250 MTR_SLACK=96 MTR_CLASS_LEAVES=1024
run k1000_s192_c1024_g1_d12500 12500 1000 MTR_SLACK=192 MTR_CLASS_LEAVES=1024 MTR_GROUPS=1
run k1000_s192_c1024_d100000 100000 1000 MTR_SLACK=192 MTR_CLASS_LEAVES=1024
run base_d100000 100000 48
echo done > $OUT/done
