#!/bin/bash
set -e
mkdir -p gpurun_out
run() { name=$1; shift; env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --steps 2 > gpurun_out/c3_$name.log 2>&1; }
run base MTR_X=0
run cl32 MTR_CLASS_LEAVES=32
run cl96 MTR_CLASS_LEAVES=96
run sl4 MTR_SLACK=4
run sl16 MTR_SLACK=16
