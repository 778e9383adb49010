#!/bin/bash
# Round-end measurements, part B: C3 kernel-trace stats + PMC passes (scripts/profile_box.sh, with the GRBM clock
# pass), then C5's, C4's and C2's kernel trace and PMC passes, each as its own rocprofv3 run.
# usage: bash scripts/round_end_b.sh <tag> [configs...]
set -e
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
TAG=${1:-r05_end}; shift || true
CFGS=${@:-C5 C4 C2}
if [ -z "$SKIP_C3" ]; then bash scripts/profile_box.sh $TAG --steps 1 --warmup 0 --no-cpu-baseline --e2e-steps 0; fi
mkdir -p gpurun_out/prof_$TAG
for cfg in $CFGS; do
  OUT=gpurun_out/prof_${TAG}_$(echo $cfg | tr A-Z a-z)
  mkdir -p $OUT
  ARGS="--config $cfg --steps 1 --warmup 0 --no-cpu-baseline --e2e-steps 0"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 -u bench.py $ARGS > $OUT/kt.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 -u bench.py $ARGS > $OUT/fetch.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 -u bench.py $ARGS > $OUT/write.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $OUT/sq -o sq --output-format csv -- python3 -u bench.py $ARGS > $OUT/sq.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_SMEM -d $OUT/sq2 -o sq2 --output-format csv -- python3 -u bench.py $ARGS > $OUT/sq2.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/grbm -o grbm --output-format csv -- python3 -u bench.py $ARGS > $OUT/grbm.log 2>&1
done
echo done > gpurun_out/prof_$TAG/done_b
