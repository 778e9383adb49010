#!/bin/bash
# More scheduling knobs: C4 ops per launch (128-leaf pair classes), C3 at 100,000 documents with 48- / 80-leaf
# classes, C2 with 192- / 256-leaf classes.  usage: bash scripts/sched_sweep2.sh <tag>
set -e
OUT=gpurun_out/sched2_${1:-r04}
mkdir -p $OUT
B="--warmup 1 --e2e-steps 0 --no-cpu-baseline"
for k in 96 192; do
  timeout -k 10 300 python3 -u bench.py --config C4 --steps 1 --ops-per-launch $k $B > $OUT/c4_k$k.json 2> $OUT/e
done
for cl in 48 80; do
  MTR_CLASS_LEAVES=$cl timeout -k 10 300 python3 -u bench.py --steps 3 $B > $OUT/c3_cl$cl.json 2> $OUT/e
done
for cl in 192 256; do
  MTR_CLASS_LEAVES=$cl timeout -k 10 300 python3 -u bench.py --config C2 --steps 2 $B > $OUT/c2_cl$cl.json 2> $OUT/e
done
echo done > $OUT/done
