#!/bin/bash
# Round-5 GPU check: a chosen pytest selection (-m gpu) then optional quick bench lines.
# usage: bash scripts/r05_gpu_check.sh <tag> "<pytest args>" [configs...]
set -e
TAG=$1; shift
SEL=$1; shift
OUT=gpurun_out/r05_$TAG
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
for c in "$@"; do
  timeout -k 10 300 python3 -u bench.py --config $c --steps 3 --warmup 1 --e2e-steps 0 --no-cpu-baseline > $OUT/$c.json 2> $OUT/$c.err
done
echo done > $OUT/done
