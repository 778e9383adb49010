#!/bin/bash
# The strong-scaling prediction of C3 on one GPU: 100,000 / N documents per GPU for N = 1, 2, 4, 8 (default
# policies), and C2 with the default and 64-leaf classes.  usage: bash scripts/strong_predict.sh <tag>
set -e
OUT=gpurun_out/strong_${1:-r04}
mkdir -p $OUT
B="--steps 3 --warmup 1 --e2e-steps 0 --no-cpu-baseline"
for d in 100000 50000 25000 12500; do
  timeout -k 10 200 python3 -u bench.py $B --docs $d > $OUT/d$d.json 2> $OUT/d$d.err
done
timeout -k 10 300 python3 -u bench.py --config C2 --steps 2 --warmup 1 --e2e-steps 0 --no-cpu-baseline > $OUT/c2.json 2> $OUT/c2.err
MTR_CLASS_LEAVES=64 timeout -k 10 300 python3 -u bench.py --config C2 --steps 2 --warmup 1 --e2e-steps 0 --no-cpu-baseline > $OUT/c2_cl64.json 2> $OUT/c2_cl64.err
echo done > $OUT/done
