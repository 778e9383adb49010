#!/bin/bash
# A/B of experiment builds on C3: per library one bench line, then the instruction-count PMC pass (one
# rocprofv3 run each).  usage: bash scripts/ab_box.sh <tag> <lib> [lib...]
set -e
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
TAG=$1; shift
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
B="--steps 3 --warmup 1 --e2e-steps 0 --no-cpu-baseline"
P="--steps 1 --warmup 0 --e2e-steps 0 --no-cpu-baseline"
for lib in "$@"; do
  MTR_LIB=$lib timeout -k 10 200 python3 -u bench.py $B > $OUT/$lib.json 2> $OUT/$lib.err
  MTR_LIB=$lib timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_SMEM -d $OUT/sq2_$lib -o sq2 --output-format csv -- python3 -u bench.py $P > $OUT/sq2_$lib.log 2>&1
done
echo done > $OUT/done
