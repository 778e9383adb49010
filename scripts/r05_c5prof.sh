#!/bin/bash
# C5-shaped phase timers on the profiling build (libmtr_prof.so).  usage: bash scripts/r05_c5prof.sh <tag> [docs]
set -e
TAG=$1
OUT=gpurun_out/r05_c5prof_$TAG
mkdir -p $OUT
MTR_LIB=libmtr_prof.so timeout -k 10 400 python3 -u scripts/phase_profile.py --docs ${2:-256} --ops ${3:-2000} --writers 64 --max-lag 4096 --grow 200000 --ops-per-launch 512 > $OUT/phase_c5.json 2> $OUT/phase_c5.err
echo done > $OUT/done
