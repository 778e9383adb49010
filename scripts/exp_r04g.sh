#!/bin/bash
# The full GPU suite on the main build, then: C4 with one vs two waves per matrix pair, C1 with 48 vs 2,048 ops per
# launch, and document groups (MTR_GROUPS 1 / 2) at 12,500 and 100,000 documents.  A test failure (exit 1) lets the
# measurements run; a time limit, abort or fault ends the script.
OUT=gpurun_out/r04g
mkdir -p $OUT
ok() { rc=$?; echo "$1 rc=$rc" >> $OUT/rc.txt; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; ok tests
B="--steps 3 --warmup 1 --e2e-steps 0 --no-cpu-baseline"
MTR_PAIR1=1 timeout -k 10 240 python3 -u bench.py --config C4 $B > $OUT/c4_pair1.json 2> $OUT/c4_pair1.err; ok c4_pair1
timeout -k 10 240 python3 -u bench.py --config C4 $B > $OUT/c4_pair2.json 2> $OUT/c4_pair2.err; ok c4_pair2
timeout -k 10 120 python3 -u bench.py --config C1 $B > $OUT/c1_k48.json 2> $OUT/c1_k48.err; ok c1_k48
timeout -k 10 120 python3 -u bench.py --config C1 $B --ops-per-launch 2048 > $OUT/c1_k2048.json 2> $OUT/c1_k2048.err; ok c1_k2048
for docs in 12500 100000; do
  for g in 1 2; do
    MTR_GROUPS=$g timeout -k 10 200 python3 -u bench.py $B --docs $docs > $OUT/d${docs}_g${g}.json 2> $OUT/d${docs}_g${g}.err; ok d${docs}_g${g}
  done
done
