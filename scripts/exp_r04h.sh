#!/bin/bash
# Spill experiment and C5: the HBM-resident parity tests on builds of the current source whose lean HBM kernel
# spills (MTR_WPE_G=5: 198 VGPRs spilled, 8: 477), the spill bisect on two commits after 428d780, then the full C5
# bench (LDS-atomic-free dirty-chunk sums) and a C5-shaped phase profile.
OUT=gpurun_out/r04h
mkdir -p $OUT
ok() { rc=$?; echo "$1 rc=$rc" >> $OUT/rc.txt; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
for lib in libmtr_spill5.so libmtr_spill8.so; do
  MTR_LIB=$lib timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -k "c5_shaped or c5_full" -v \
    --timeout 300 --timeout-method thread > $OUT/$lib.log 2>&1; ok $lib
done
for c in old_1a5aea1 old_cfbc877; do
  (cd gpurun_exp/$c && MTR_LIB=libmtr_s5.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "c5_shaped" -v \
     --timeout 250 --timeout-method thread) > $OUT/$c.log 2>&1; ok $c
done
timeout -k 10 400 python3 -u bench.py --config C5 --steps 1 --warmup 1 --e2e-steps 0 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err; ok c5
MTR_LIB=libmtr_prof.so timeout -k 10 300 python3 -u scripts/phase_profile.py --docs 256 --ops 2000 --writers 64 --max-lag 4096 --grow 200000 --ops-per-launch 512 > $OUT/phase_c5.json 2> $OUT/phase_c5.err; ok phase_c5
MTR_LIB=libmtr_prof.so timeout -k 10 300 python3 -u scripts/phase_profile.py --docs 20000 > $OUT/phase_c3.json 2> $OUT/phase_c3.err; ok phase_c3
