#!/bin/bash
# GPU parity suite, then quick bench lines.  usage: bash scripts/gpu_check.sh <tag> [configs...]
set -e
TAG=${1:-check}; shift || true
OUT=gpurun_out/check_$TAG
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
for c in "$@"; do
  timeout -k 10 300 python3 -u bench.py --config $c --steps 3 --warmup 1 --e2e-steps 0 --no-cpu-baseline > $OUT/$c.json 2> $OUT/$c.err
done
