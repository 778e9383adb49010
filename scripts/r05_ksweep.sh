#!/bin/bash
# ops-per-launch sweep for C2 / C4 (launch count vs per-launch tail).  usage: bash scripts/r05_ksweep.sh <tag>
set -e
OUT=gpurun_out/r05_ksweep_$1
mkdir -p $OUT
for cfg in ${CFGS:-C4 C2}; do
  for k in ${KS:-48 96 192}; do
    timeout -k 10 300 python3 -u bench.py --config $cfg --steps 2 --warmup 1 --e2e-steps 0 --no-cpu-baseline --ops-per-launch $k > $OUT/${cfg}_k$k.json 2> $OUT/${cfg}_k$k.err
  done
done
echo done > $OUT/done
