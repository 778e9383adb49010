#!/bin/bash
# one config under a list of env settings.  usage: bash scripts/r05_knobs.sh <tag> <config> "<ENV=VAL>" ...
set -e
OUT=gpurun_out/r05_knobs_$1
mkdir -p $OUT
CFG=$2; shift 2
for kv in "$@"; do
  n=$(echo "$kv" | tr '= ' '__')
  env $kv timeout -k 10 300 python3 -u bench.py --config $CFG --steps 2 --warmup 1 --e2e-steps 0 --no-cpu-baseline > $OUT/${CFG}_$n.json 2> $OUT/${CFG}_$n.err
done
echo done > $OUT/done
