#!/bin/bash
# C2 / C3 bench lines plus the LDS parity tests on the current build.  usage: bash scripts/r05_c2c3.sh <tag>
set -e
OUT=gpurun_out/r05_c2c3_$1
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || (echo "tests rc=$?" >> $OUT/tests.log; exit 1)
for cfg in C2 C3; do
  timeout -k 10 300 python3 -u bench.py --config $cfg --steps 2 --warmup 1 --e2e-steps 0 > $OUT/$cfg.json 2> $OUT/$cfg.err
done
echo done > $OUT/done
