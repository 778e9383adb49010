#!/bin/bash
# Kernel-trace + PMC passes of one config's bench (as scripts/round_end_b.sh does for C5 / C4), each pass its own
# rocprofv3 run.  usage: bash scripts/profile_cfg.sh <tag> <config>
set -e
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
TAG=$1; cfg=$2
OUT=gpurun_out/prof_${TAG}_$(echo $cfg | tr A-Z a-z)
mkdir -p $OUT
ARGS="--config $cfg --steps 1 --warmup 0 --no-cpu-baseline --e2e-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 -u bench.py $ARGS > $OUT/kt.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 -u bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 -u bench.py $ARGS > $OUT/write.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $OUT/sq -o sq --output-format csv -- python3 -u bench.py $ARGS > $OUT/sq.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_SMEM -d $OUT/sq2 -o sq2 --output-format csv -- python3 -u bench.py $ARGS > $OUT/sq2.log 2>&1
echo done > $OUT/done
