#!/bin/bash
# Spill bisect (commits after 428d780 built with -DMTR_WPE_G=5), then the deferred merge-copy build (vp3): its
# GPU suite and its A/B against the main build.  Ordinary failures (exit 1) let the next step run.
OUT=gpurun_out/r04e
mkdir -p $OUT
ok() { rc=$?; echo "$1 rc=$rc" >> $OUT/rc.txt; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
for c in old_1a5aea1 old_cfbc877; do
  (cd gpurun_exp/$c && MTR_LIB=libmtr_s5.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -k "c5_shaped" -v \
     --timeout 300 --timeout-method thread) > $OUT/$c.log 2>&1; ok $c
done
MTR_LIB=libmtr_main4.so timeout -k 10 700 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_main4.log 2>&1; ok tests_main4
bash scripts/ab_box.sh r04e libmtr.so libmtr_main4.so; ok ab
