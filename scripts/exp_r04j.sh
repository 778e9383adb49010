#!/bin/bash
# The spill experiment's insert placement: the C5-shaped documents up to their first divergent op on the
# MTR_WPE_G=8 build and on a spill-free one, both printing each insert's placement (-DMTR_DEBUG_INSERT); then the
# main build (bounded view scan, fused parent-block walk, batched record updates, two document groups by
# default): the GPU suite, C3 at 100,000 and 12,500 documents, C5.
OUT=gpurun_out/r04j
mkdir -p $OUT
ok() { rc=$?; echo "$1 rc=$rc" >> $OUT/rc.txt; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
MTR_LIB=libmtr_spill8dbg.so timeout -k 10 300 python3 -u scripts/probes/ins_debug.py > $OUT/ins_spill8.log 2>&1; ok ins_spill8
MTR_LIB=libmtr_dbg.so timeout -k 10 300 python3 -u scripts/probes/ins_debug.py > $OUT/ins_nospill.log 2>&1; ok ins_nospill
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; ok tests
B="--steps 3 --warmup 1 --e2e-steps 0 --no-cpu-baseline"
timeout -k 10 300 python3 -u bench.py $B > $OUT/c3.json 2> $OUT/c3.err; ok c3
timeout -k 10 200 python3 -u bench.py $B --docs 12500 > $OUT/c3_12500.json 2> $OUT/c3_12500.err; ok c3_12500
timeout -k 10 400 python3 -u bench.py --config C5 --steps 1 --warmup 1 --e2e-steps 0 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err; ok c5
