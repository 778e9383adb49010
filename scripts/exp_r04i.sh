#!/bin/bash
# The combining / interval GPU tests after the empty-property-set fix; HBM-resident parity and C5 on the build with
# the bounded two-level view scan, fused parent-block walk and batched record updates (libmtr_vb.so) and on the main
# build; the document-group policy sweep (C3 shares, C2); the spill8 bisect.
OUT=gpurun_out/r04i
mkdir -p $OUT
ok() { rc=$?; echo "$1 rc=$rc" >> $OUT/rc.txt; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
timeout -k 10 300 python3 -u -m pytest tests/test_local_combining.py tests/test_intervals.py -m gpu -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1; ok tests
MTR_LIB=libmtr_vb.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -k "c5_shaped or c5_full" -q --timeout 300 --timeout-method thread > $OUT/gpu_c5_tests_vb.log 2>&1; ok c5_tests_vb
MTR_LIB=libmtr_vb.so timeout -k 10 400 python3 -u bench.py --config C5 --steps 1 --warmup 1 --e2e-steps 0 --no-cpu-baseline > $OUT/c5_vb.json 2> $OUT/c5_vb.err; ok c5_vb
timeout -k 10 400 python3 -u bench.py --config C5 --steps 1 --warmup 1 --e2e-steps 0 --no-cpu-baseline > $OUT/c5_main.json 2> $OUT/c5_main.err; ok c5_main
B="--steps 3 --warmup 1 --e2e-steps 0 --no-cpu-baseline"
for docs in 12500 25000 50000; do
  for g in 2 3 4; do
    MTR_GROUPS=$g timeout -k 10 200 python3 -u bench.py $B --docs $docs > $OUT/d${docs}_g${g}.json 2> $OUT/d${docs}_g${g}.err; ok d${docs}_g${g}
  done
done
for g in 1 2 3; do
  MTR_GROUPS=$g timeout -k 10 300 python3 -u bench.py --config C2 $B > $OUT/c2_g${g}.json 2> $OUT/c2_g${g}.err; ok c2_g${g}
done
MTR_LIB=libmtr_spill8.so timeout -k 10 300 python3 -u scripts/probes/c5_bisect.py > $OUT/bisect_spill8.log 2>&1; ok bisect_spill8
