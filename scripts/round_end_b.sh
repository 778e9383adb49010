#!/bin/bash
# Round-end measurements, part B: C3 kernel-trace stats + PMC passes (scripts/profile_box.sh), then C5's and C4's
# kernel trace and PMC passes, each as its own rocprofv3 run.
set -e
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
TAG=${1:-r04_end}
bash scripts/profile_box.sh $TAG --steps 1 --warmup 0 --no-cpu-baseline --e2e-steps 0
for cfg in C5 C4; do
  OUT=gpurun_out/prof_${TAG}_$(echo $cfg | tr A-Z a-z)
  mkdir -p $OUT
  ARGS="--config $cfg --steps 1 --warmup 0 --no-cpu-baseline --e2e-steps 0"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 -u bench.py $ARGS > $OUT/kt.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 -u bench.py $ARGS > $OUT/fetch.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 -u bench.py $ARGS > $OUT/write.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $OUT/sq -o sq --output-format csv -- python3 -u bench.py $ARGS > $OUT/sq.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_SMEM -d $OUT/sq2 -o sq2 --output-format csv -- python3 -u bench.py $ARGS > $OUT/sq2.log 2>&1
done
echo done > gpurun_out/prof_$TAG/done_b
# phase timers (libmtr_prof.so: -DMTR_PROF) on C3- and C5-shaped batches
MTR_LIB=libmtr_prof.so timeout -k 10 300 python3 -u scripts/phase_profile.py --docs 20000 > gpurun_out/prof_$TAG/phase_c3.json 2>&1
MTR_LIB=libmtr_prof.so timeout -k 10 300 python3 -u scripts/phase_profile.py --docs 256 --ops 2000 --writers 64 --max-lag 4096 --grow 200000 --ops-per-launch 512 > gpurun_out/prof_$TAG/phase_c5.json 2>&1
# launch granularity at the 8-GPU share with two groups
for k in 96 192; do
  timeout -k 10 200 python3 -u bench.py --steps 3 --warmup 1 --e2e-steps 0 --no-cpu-baseline --docs 12500 --ops-per-launch $k > gpurun_out/prof_$TAG/c3_12500_k$k.json 2>&1
done
