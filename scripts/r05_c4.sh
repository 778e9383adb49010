#!/bin/bash
# C4 on the current build: the matrix parity tests, then the C4 bench line.  usage: bash scripts/r05_c4.sh <tag>
set -e
OUT=gpurun_out/r05_c4_$1
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_matrix.py tests/test_gpu_parity.py tests/test_matrix_undo.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
timeout -k 10 300 python3 -u bench.py --config C4 --steps 2 --warmup 1 --e2e-steps 0 --no-cpu-baseline > $OUT/C4.json 2> $OUT/C4.err
echo done > $OUT/done
