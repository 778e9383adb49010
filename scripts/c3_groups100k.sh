#!/bin/bash
# C3 at 100,000 documents: one document group (default above 60,000) against two, alternating, three runs each.
set -e
OUT=gpurun_out/g100k_${1:-r04}
mkdir -p $OUT
B="--steps 5 --warmup 1 --e2e-steps 0 --no-cpu-baseline"
for r in 1 2 3; do
  MTR_GROUPS=1 timeout -k 10 200 python3 -u bench.py $B > $OUT/g1_$r.json 2> $OUT/e
  MTR_GROUPS=2 timeout -k 10 200 python3 -u bench.py $B > $OUT/g2_$r.json 2> $OUT/e
done
echo done > $OUT/done
