#!/bin/bash
# C3 issue-side experiment on one build: bench lines with the launch knobs (MTR_LANES, MTR_NO_FIXED_CAP),
# then PMC passes for the instruction cache and the per-unit issue cycles (each its own rocprofv3 run).
# usage: bash scripts/issue_box.sh <tag> [lib]
set -e
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
TAG=${1:-r04}
export MTR_LIB=${2:-libmtr.so}
OUT=gpurun_out/issue_$TAG
mkdir -p $OUT
B="--steps 3 --warmup 1 --e2e-steps 0 --no-cpu-baseline"
timeout -k 10 200 python3 -u bench.py $B > $OUT/c3.json 2> $OUT/c3.err
MTR_LANES=1 timeout -k 10 200 python3 -u bench.py $B > $OUT/c3_lanes1.json 2> $OUT/c3_lanes1.err
MTR_NO_FIXED_CAP=1 timeout -k 10 200 python3 -u bench.py $B > $OUT/c3_nofixed.json 2> $OUT/c3_nofixed.err
P="--steps 1 --warmup 0 --e2e-steps 0 --no-cpu-baseline"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 -u bench.py $P > $OUT/kt.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ -d $OUT/ic -o ic --output-format csv -- python3 -u bench.py $P > $OUT/ic.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_ANY -d $OUT/sq3 -o sq3 --output-format csv -- python3 -u bench.py $P > $OUT/sq3.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_SMEM -d $OUT/sq2 -o sq2 --output-format csv -- python3 -u bench.py $P > $OUT/sq2.log 2>&1
echo done > $OUT/done
