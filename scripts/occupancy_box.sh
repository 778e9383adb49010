#!/bin/bash
# Occupancy / issue PMC passes of the C3 bench (one rocprofv3 run per pass, each under its own limit)
# usage: bash scripts/occupancy_box.sh <tag> [lib]
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
TAG=${1:-r02}; LIB=${2:-libmtr.so}
OUT=gpurun_out/occ_$TAG
mkdir -p $OUT
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --e2e-steps 0"
export MTR_LIB=$LIB
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 -u bench.py $ARGS > $OUT/kt.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc MeanOccupancyPerCU -d $OUT/occ -o occ --output-format csv -- python3 -u bench.py $ARGS > $OUT/occ.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc SALUBusy -d $OUT/salu -o salu --output-format csv -- python3 -u bench.py $ARGS > $OUT/salu.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES -d $OUT/sq -o sq --output-format csv -- python3 -u bench.py $ARGS > $OUT/sq.log 2>&1
rc=$?
find $OUT -name '*.csv' | sort
exit $rc
