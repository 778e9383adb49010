#!/bin/bash
# document-group A/B (MTR_GROUPS) for one config.  usage: bash scripts/r05_groups.sh <tag> <config> [groups...]
set -e
OUT=gpurun_out/r05_groups_$1
mkdir -p $OUT
CFG=$2; shift 2
for g in ${@:-1 2 3 4}; do
  MTR_GROUPS=$g timeout -k 10 300 python3 -u bench.py --config $CFG --steps 2 --warmup 1 --e2e-steps 0 --no-cpu-baseline > $OUT/${CFG}_g$g.json 2> $OUT/${CFG}_g$g.err
done
echo done > $OUT/done
