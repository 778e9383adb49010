#!/bin/bash
# C3 (100,000 documents) launch knobs on the final build: slack leaves per document (MTR_SLACK) and ops per launch.
set -e
OUT=gpurun_out/c3k_${1:-r04}
mkdir -p $OUT
B="--steps 3 --warmup 1 --e2e-steps 0 --no-cpu-baseline"
timeout -k 10 200 python3 -u bench.py $B > $OUT/base.json 2> $OUT/e
for sl in 4 16 24; do MTR_SLACK=$sl timeout -k 10 200 python3 -u bench.py $B > $OUT/slack$sl.json 2> $OUT/e; done
for k in 40 56; do timeout -k 10 200 python3 -u bench.py $B --ops-per-launch $k > $OUT/k$k.json 2> $OUT/e; done
echo done > $OUT/done
