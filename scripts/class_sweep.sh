#!/bin/bash
# Size-class width (MTR_CLASS_LEAVES) at the 8-GPU share of C3 (12,500 documents, two groups): narrower classes
# make a launch's documents more alike in cost (less tail per round), at more launches per round.
set -e
OUT=gpurun_out/class_${1:-r04}
mkdir -p $OUT
B="--steps 3 --warmup 1 --e2e-steps 0 --no-cpu-baseline --docs 12500"
for cl in 32 48 64 96; do
  MTR_CLASS_LEAVES=$cl timeout -k 10 200 python3 -u bench.py $B > $OUT/cl$cl.json 2> $OUT/cl$cl.err
done
echo done > $OUT/done
