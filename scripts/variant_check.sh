#!/bin/bash
# One engine build on C3: the bench line (3 timed steps) and one PMC pass of instruction counts.
# usage: bash scripts/variant_check.sh <tag> [MTR_LIB]   (e.g. libmtr_v23.so built by build.py --variant v23)
set -e
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
TAG=${1:-v}; LIBNAME=${2:-libmtr.so}
OUT=gpurun_out/var_$TAG
mkdir -p $OUT
MTR_LIB=$LIBNAME timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --e2e-steps 0 --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err
MTR_LIB=$LIBNAME timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_SMEM -d $OUT/sq2 -o sq2 --output-format csv -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --e2e-steps 0 > $OUT/sq2.log 2>&1
