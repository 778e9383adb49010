#!/bin/bash
# Every document of C3 and C5 checked against the oracle (the bench's sample widened to the whole batch).
# usage: bash scripts/r05_fullcheck.sh <tag>
set -e
OUT=gpurun_out/full_$1
mkdir -p $OUT
if [ -z "$SKIP_C3" ]; then
timeout -k 10 400 python3 -u bench.py --config C3 --steps 1 --warmup 1 --e2e-steps 0 --cpu-sample-docs 100000 > $OUT/c3.json 2> $OUT/c3.err
fi
# (the C5 check is minutes of silent host work: a heartbeat file keeps the box's hang detector informed)
( while sleep 50; do date >> $OUT/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 800 python3 -u bench.py --config C5 --steps 1 --warmup 0 --cpu-sample-docs 1000 > $OUT/c5.json 2> $OUT/c5.err
echo done > $OUT/done
