#!/bin/bash
# The spill experiment: the C5-shaped parity case on the MTR_WPE_G=8 build (libmtr_wpeg8.so,
# -DMTR_DEBUG_INSERT prints each insert's placement).  usage: bash scripts/r05_spill.sh <tag> [lib]
set -e
OUT=gpurun_out/r05_spill_$1
mkdir -p $OUT
MTR_LIB=${2:-libmtr_wpeg8.so} timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -k "c5_shaped and 20k-segments and not long" -x -q --timeout 360 --timeout-method thread > $OUT/test.log 2>&1 || echo "rc=$?" >> $OUT/test.log
echo done > $OUT/done
