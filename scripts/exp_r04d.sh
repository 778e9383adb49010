#!/bin/bash
# GPU suite on the main build; the round-3 spill failure reproduced on commit 428d780's source built to spill
# (gpurun_exp/old428, -DMTR_WPE_G=5); the launch knobs and instruction-cache counters; the launch-policy sweep.
# Ordinary failures (exit 1) let the next step run; anything else ends the script.
OUT=gpurun_out/r04d
mkdir -p $OUT
ok() { rc=$?; echo "$1 rc=$rc" >> $OUT/rc.txt; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; ok tests
(cd gpurun_exp/old428 && MTR_LIB=libmtr_s5.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -k "c5_shaped" -v \
   --timeout 300 --timeout-method thread) > $OUT/old428_s5.log 2>&1; ok old428
bash scripts/icache_box.sh r04d; ok icache
bash scripts/launch_sweep.sh r04d; ok sweep
