#!/bin/bash
# Round profile on the GPU box: kernel-trace stats of the bench command, then one PMC pass per
# counter group (HBM bytes, LDS banking, wave-state), each as its own rocprofv3 run.
# usage: bash scripts/profile_box.sh <tag> [bench args...]
set -e
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
TAG=${1:-r01}; shift || true
ARGS=${@:---steps 1 --warmup 0 --no-cpu-baseline}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 -u bench.py $ARGS > $OUT/kt.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 -u bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 -u bench.py $ARGS > $OUT/write.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $OUT/sq -o sq --output-format csv -- python3 -u bench.py $ARGS > $OUT/sq.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_SMEM -d $OUT/sq2 -o sq2 --output-format csv -- python3 -u bench.py $ARGS > $OUT/sq2.log 2>&1
# the shader clock the kernels ran at: GRBM_GUI_ACTIVE (summed over the 8 XCDs) / 8 / dispatch duration
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/grbm -o grbm --output-format csv -- python3 -u bench.py $ARGS > $OUT/grbm.log 2>&1
find $OUT -name '*.csv' | sort
