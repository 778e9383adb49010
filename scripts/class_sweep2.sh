#!/bin/bash
# Size-class width (MTR_CLASS_LEAVES) at the strong-scaling shares of C3 (100,000 / N documents per GPU).
set -e
OUT=gpurun_out/class2_${1:-r04}
mkdir -p $OUT
B="--steps 3 --warmup 1 --e2e-steps 0 --no-cpu-baseline"
for cl in 128 160 192; do
  MTR_CLASS_LEAVES=$cl timeout -k 10 200 python3 -u bench.py $B --docs 12500 > $OUT/d12500_cl$cl.json 2> $OUT/e1
done
for d in 25000 50000 100000; do
  for cl in 64 96 128; do
    MTR_CLASS_LEAVES=$cl timeout -k 10 200 python3 -u bench.py $B --docs $d > $OUT/d${d}_cl$cl.json 2> $OUT/e2
  done
done
echo done > $OUT/done
