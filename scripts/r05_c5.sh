#!/bin/bash
# C5 on the team build: the HBM-resident parity tests, then C5 bench lines.
# usage: bash scripts/r05_c5.sh <tag> [bench steps]
set -e
TAG=$1
OUT=gpurun_out/r05_c5_$TAG
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -k "c5" -x -v --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1
timeout -k 10 600 python3 -u bench.py --config C5 --steps ${2:-1} --warmup 0 --e2e-steps 0 --no-cpu-baseline > $OUT/C5.json 2> $OUT/C5.err
echo done > $OUT/done
