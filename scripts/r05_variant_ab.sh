#!/bin/bash
# C3 / C2 A/B of experiment builds (libmtr_<name>.so, selected with MTR_LIB) against the main build.
# usage: bash scripts/r05_variant_ab.sh <tag> <name>...
set -e
OUT=gpurun_out/vab_$1; shift
mkdir -p $OUT
B="--steps 2 --warmup 1 --e2e-steps 0"
for v in main "$@"; do
  lib=libmtr.so; [ $v != main ] && lib=libmtr_$v.so
  for cfg in C3 C2; do
    MTR_LIB=$lib timeout -k 10 300 python3 -u bench.py --config $cfg $B > $OUT/${cfg}_$v.json 2> $OUT/${cfg}_$v.err
  done
done
echo done > $OUT/done
