#!/bin/bash
# Round-4 experiment set: GPU suite on the main build, the spill experiment, then A/B of the VALU-predicate
# builds.  A step that fails with an ordinary error (exit 1) lets the next run; a time limit, abort, fault or
# crash (any other status) ends the script.
OUT=gpurun_out/r04c
mkdir -p $OUT
ok() { rc=$?; echo "$1 rc=$rc" >> $OUT/rc.txt; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; ok tests
bash scripts/spill_box.sh r04c; ok spill
bash scripts/ab_box.sh r04c libmtr.so libmtr_vp.so libmtr_vp2.so; ok ab
