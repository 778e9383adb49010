#!/bin/bash
# Scheduling knobs on the other configs: C4's class width (matrix pairs), C2's ops per launch with 128-leaf
# classes, C1's class width.  usage: bash scripts/sched_sweep.sh <tag>
set -e
OUT=gpurun_out/sched_${1:-r04}
mkdir -p $OUT
B="--warmup 1 --e2e-steps 0 --no-cpu-baseline"
for cl in 128 256 512; do
  MTR_CLASS_LEAVES=$cl timeout -k 10 300 python3 -u bench.py --config C4 --steps 1 $B > $OUT/c4_cl$cl.json 2> $OUT/e
done
for k in 64 96; do
  timeout -k 10 300 python3 -u bench.py --config C2 --steps 2 --ops-per-launch $k $B > $OUT/c2_k$k.json 2> $OUT/e
done
for cl in 128 256; do
  MTR_CLASS_LEAVES=$cl timeout -k 10 300 python3 -u bench.py --config C1 --steps 5 $B > $OUT/c1_cl$cl.json 2> $OUT/e
done
echo done > $OUT/done
