#!/bin/bash
# The full GPU suite on the main build (interval collections; the round loop in document groups, one group by
# default), then the document-group sweep at the strong-scaling shares.  A test failure (exit 1) lets the sweep run.
OUT=gpurun_out/r04g
mkdir -p $OUT
ok() { rc=$?; echo "$1 rc=$rc" >> $OUT/rc.txt; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; ok tests
bash scripts/groups_sweep.sh r04g; ok groups
