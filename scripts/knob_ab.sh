#!/bin/bash
# C3 launch-policy A/B on one box (device-resident bench lines, no CPU leg): the default, then each knob.
# usage: bash scripts/knob_ab.sh <tag> "<ENV=VAL [bench args]>" ...
TAG=$1; shift
OUT=gpurun_out/knobs_$TAG
mkdir -p $OUT
i=0
timeout -k 10 300 python3 -u bench.py --steps 5 --e2e-steps 0 --no-cpu-baseline > $OUT/base.json 2> $OUT/base.err || exit $?
for spec in "$@"; do
  i=$((i+1))
  echo "$spec" > $OUT/k$i.spec
  env $(echo "$spec" | tr ' ' '\n' | grep '=' | tr '\n' ' ') timeout -k 10 300 python3 -u bench.py --steps 5 --e2e-steps 0 --no-cpu-baseline $(echo "$spec" | tr ' ' '\n' | grep -v '=' | tr '\n' ' ') > $OUT/k$i.json 2> $OUT/k$i.err || exit $?
done
timeout -k 10 300 python3 -u bench.py --steps 5 --e2e-steps 0 --no-cpu-baseline > $OUT/base2.json 2> $OUT/base2.err
