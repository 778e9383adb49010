#!/bin/bash
# Parity sweep on the GPU box: bench runs off the presets' shapes (writers, lag, ops per launch, document
# sizes), each checking its sampled documents against the oracle bit for bit.  A failing run ends the script.
# (the synthetic generator takes up to 64 writers, MTR_SYNTH_MAX_WRITERS)
# usage: [ONLY=<regex of run names>] bash scripts/r05_stress.sh <tag>;  summary: python3 scripts/stress_summary.py gpurun_out/stress_<tag>
set -e
OUT=gpurun_out/stress_$1
mkdir -p $OUT
run() {  # name, bench args...
  local name=$1; shift
  if [ -n "$ONLY" ] && ! [[ $name =~ $ONLY ]]; then return 0; fi
  timeout -k 10 240 python3 -u bench.py --steps 1 --warmup 0 --e2e-steps 0 "$@" \
    > $OUT/$name.json 2> $OUT/$name.err
}
run c2_w2_lag0 --config C2 --docs 2000 --writers 2 --max-lag 0
run c2_w64_lag512 --config C2 --docs 2000 --writers 64 --max-lag 512
run c2_w64_lag4096 --config C2 --docs 1000 --writers 64 --max-lag 4096
run c2_k1 --config C2 --docs 1000 --ops 600 --ops-per-launch 1
run c2_k7 --config C2 --docs 2000 --ops-per-launch 7
run c2_k500 --config C2 --docs 2000 --ops-per-launch 500
run c3_w32_lag256 --config C3 --docs 20000 --writers 32 --max-lag 256
run c3_ops8000 --config C3 --docs 4000 --ops 8000
run c4_w32_lag512 --config C4 --docs 400 --writers 32 --max-lag 512
run c4_k5 --config C4 --docs 400 --ops 4000 --ops-per-launch 5
run c5_w8_lag64 --config C5 --docs 64 --ops 4000 --writers 8 --max-lag 64
run c5_w64_lag8192 --config C5 --docs 64 --ops 4000 --writers 64 --max-lag 8192
echo done > $OUT/done
