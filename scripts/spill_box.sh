#!/bin/bash
# The spill experiment: the HBM-resident parity tests on builds whose lean HBM kernel
# spills VGPRs to scratch (-DMTR_WPE_G=4), without (libmtr_spillA.so) and with (libmtr_spillB.so) a fix.
# A failing pytest (exit 1) goes on to the next build; a time limit, abort or fault ends the script.
# usage: bash scripts/spill_box.sh <tag> [libs...]
TAG=${1:-r04}; shift || true
LIBS=${@:-libmtr_spillA.so libmtr_spillB.so}
OUT=gpurun_out/spill_$TAG
mkdir -p $OUT
for lib in $LIBS; do
  MTR_LIB=$lib timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -k "c5_shaped or c5_full" -v \
    --timeout 300 --timeout-method thread > $OUT/$lib.log 2>&1
  rc=$?
  echo "$lib rc=$rc" >> $OUT/rc.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
exit 0
