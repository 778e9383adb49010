#!/bin/bash
# Round-4 check: the spill bisect (two commits after 428d780 built with -DMTR_WPE_G=5), the full GPU suite on the
# main build (deferred merge copy, local combining, interval collections), then the A/B of the previous main build
# (libmtr_vp2.so) against it.  Ordinary test failures (exit 1) let the next step run.
OUT=gpurun_out/r04f
mkdir -p $OUT
ok() { rc=$?; echo "$1 rc=$rc" >> $OUT/rc.txt; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; ok tests
for c in old_1a5aea1 old_cfbc877; do
  (cd gpurun_exp/$c && MTR_LIB=libmtr_s5.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -k "c5_shaped" -v \
     --timeout 300 --timeout-method thread) > $OUT/$c.log 2>&1; ok $c
done
bash scripts/ab_box.sh r04f libmtr_vp2.so libmtr.so; ok ab
