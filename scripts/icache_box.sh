#!/bin/bash
# Launch knobs (MTR_LANES, MTR_NO_FIXED_CAP) on C3 and the instruction-cache counters of the default build.
# usage: bash scripts/icache_box.sh <tag>
set -e
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=gpurun_out/issue_${1:-r04}
mkdir -p $OUT
B="--steps 3 --warmup 1 --e2e-steps 0 --no-cpu-baseline"
P="--steps 1 --warmup 0 --e2e-steps 0 --no-cpu-baseline"
MTR_LANES=1 timeout -k 10 200 python3 -u bench.py $B > $OUT/c3_lanes1.json 2> $OUT/c3_lanes1.err
MTR_NO_FIXED_CAP=1 timeout -k 10 200 python3 -u bench.py $B > $OUT/c3_nofixed.json 2> $OUT/c3_nofixed.err
timeout -s KILL 240 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ -d $OUT/ic -o ic --output-format csv -- python3 -u bench.py $P > $OUT/ic.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_ANY -d $OUT/sq3 -o sq3 --output-format csv -- python3 -u bench.py $P > $OUT/sq3.log 2>&1
echo done > $OUT/done
